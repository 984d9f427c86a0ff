// Fused message_layer_1 kernel (see msg_pre.h for the algorithm and data layout).
#include <cstdlib>

#include "msg_pre.h"
#include "tp16.h"

namespace nbx {

constexpr int MP_THREADS = 512;
// one exchange buffer: [4 planes][6 parts][16 rows][MP_RS], 16 channels per row padded to 20
// floats so the GEMM waves' stores (lane quarters qd = 0/1 hold rows 4 apart) hit different
// bank halves, while rows stay 16-byte aligned for the edge waves' ds_read_b128
// (X3: rows unpadded, 16 floats, so that two buffers fit beside the larger bf16x3 images; the
// channel quads of row r are stored XOR-swizzled by (r >> 2) & 3 instead, which keeps the GEMM
// waves' stores -- lane quarters hold rows 4 apart -- on distinct banks and the edge waves'
// float4 reads whole)
template <bool X3> struct MpEx {   // X3: any split-precision node GEMM (bf16x3 or fp16x2)
    static constexpr int RS = X3 ? 16 : 20, PART = 16 * RS, EX = 4 * 6 * PART;
};
// exchange buffers: three beside the fp16x2 images (decoupled hand-off), two otherwise
constexpr int mp_nbuf(int prec) { return prec == 2 ? 3 : 2; }

// X3: the node GEMM on the split-precision path (tp_fused.h StatSKX3; bf16x3 CW = 16 images,
// v_mfma_f32_16x16x32_bf16 whose A fragment -- lane quarter qd holds k = 8 qd + j -- is exactly
// the X chunk a lane loads)
// (X3 runs a static schedule over KCT = ceil(M / 32) K chunks)
// (PREC 2: the fp16x2 images and v_mfma_f32_16x16x32_f16, 3 terms instead of 6; the node GEMM
// results are descaled by P.bscale as they are parked in the exchange)
// CHK (NBX_MP_CHECK=1, diagnosis builds of the hand-off; tests/test_gpu_segnn_paths.py): every wave
// checks the stage tag of the exchange buffer it is about to consume -- the group the four GEMM waves
// last wrote into it (edge waves) or the group the four edge waves last read from it (GEMM waves) --
// against the group its counters promised, and counts / printfs each mismatch (block, wave, group).
// CHK 2 also drops the edge waves' wait (fault injection: shows the check detects a broken hand-off).
template <int PREC, int KCT = 0, int CHK = 0>
__global__ __launch_bounds__(MP_THREADS, PREC ? 1 : 2) void msg_pre_kernel(const MsgPreProb P) {
    constexpr bool X3 = PREC != 0;
    // fp16x2 (images the fp32 size): three exchange buffers fit, and the two roles hand them over
    // through LDS counters instead of a block barrier per stage (DEC): the GEMM waves may run up to
    // two groups ahead of the edge waves, so per-stage jitter of either role is absorbed
    constexpr int NBUF = mp_nbuf(PREC);
#ifndef NBX_MP_DEC
#define NBX_MP_DEC 1   // 0: block barriers per stage (A/B builds only)
#endif
    constexpr bool DEC = NBX_MP_DEC && NBUF > 2;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int F = P.img_floats, M = P.M, N = P.N, G = P.G, NG = P.NG;
    constexpr int MP_RS = MpEx<X3>::RS, MP_PART = MpEx<X3>::PART, MP_EX = MpEx<X3>::EX;
    float* EX = lds + 2 * F;   // [NBUF buffers][MP_EX]
    float* XC = EX + NBUF * MP_EX;  // pending BN of X per k: [sc_s | sc_v | sh] x (KC * 32), zero past M
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63, c16 = lane & 15, qd = lane >> 4;
    const bool gemm_wave = wave < 4;
    const int plane = wave & 3;
    const unsigned long long c_start = P.dbg ? clock64() : 0ull;
    // XCD-aware block order (P.xcd_group): consecutive block ids go to different XCDs (round robin
    // over 8), so block b runs on XCD b % 8; the `chunks` blocks that share a node slab pblk are
    // given ids with the same b % 8, so the slab's X rows are fetched into one XCD's L2 once and
    // hit there for the other chunks (instead of one L2 miss stream per chunk)
    int chunk, pblk;
    if (P.xcd_group) {
        const int xcd = blockIdx.x & 7, s = blockIdx.x >> 3;
        chunk = s % P.chunks;
        pblk = (s / P.chunks) * 8 + xcd;
    } else {
        chunk = blockIdx.x % P.chunks;
        pblk = blockIdx.x / P.chunks;
    }
    const int my_groups = pblk < P.n_slabs ? (P.n_slabs - 1 - pblk) / P.per_chunk + 1 : 0;
    const int KC = (M + 31) >> 5;
    const int lg = __builtin_ctz((unsigned)G);
    const float invN = 1.0f / (float)N;
    const int64_t Ep = P.V * G;
    // M1S / M1V: 16-B buffer stores, write-through (sc1: the 39 MB edge operand leaves L2 as it is
    // written, no end-of-kernel write-back; tp_fused.h st_out; r05 A/B +1.1 % steps/s, profiles/r05/wtdv)
    const __amdgpu_buffer_rsrc_t rsS = __builtin_amdgcn_make_buffer_rsrc((void*)P.M1S, (short)0, 0x7FFFFFF0, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsV = __builtin_amdgcn_make_buffer_rsrc((void*)P.M1V, (short)0, 0x7FFFFFF0, 0x00020000);
    auto st4 = [&](const __amdgpu_buffer_rsrc_t& rs, uint32_t off, float4 v) {
        typedef unsigned v4u __attribute__((ext_vector_type(4)));
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), rs, off, 0, 16);
    };

    // GEMM waves: A = X[plane][node][k], two float4 per lane per 32-deep chunk (lane quarter qd
    // supplies k = 8 qd + s at MFMA step s), bounds-checked buffer loads (zeros past M / V)
    const __amdgpu_buffer_rsrc_t rsX = __builtin_amdgcn_make_buffer_rsrc((void*)P.X, (short)0, 0x7FFFFFF0, 0x00020000);
    auto load_a = [&](int i, int kc, float4 (&a)[2]) {
        const int grp = pblk + i * P.per_chunk;
        const int64_t node = (int64_t)grp * NG + c16;
        const int k = kc * 32 + 8 * qd;
        const bool ok = i < my_groups && c16 < NG && node < P.V && k < M;
        const uint32_t off = ok ? (uint32_t)((((int64_t)plane * P.V + node) * M + k) * 4) : 0x7FFFFFF0u;
        a[0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsX, off, 0, 0));
        a[1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rsX, ok ? off + 16 : off, 0, 0));
    };
    constexpr int KCMAX = 4;   // M <= 128 (launch check)
    float4 abuf[KCMAX][2];
    if (gemm_wave) {
#pragma unroll
        for (int kc = 0; kc < KCMAX; ++kc)
            if (kc < KC) load_a(0, kc, abuf[kc]);
    }

    // the previous layer's feature BatchNorm, finalised here from its sums: the inputs of one
    // evaluation per thread (t < 2M: kind = t / M) are loaded before the image DMA, so the
    // coefficient math waits for them only (vmcnt retires in issue order)
    const bool bn_on = P.xbn.sums != nullptr && t < 2 * M;
    const int bn_kind = t / M, bn_k = t % M;
    const BnPre bn_pre = bn_pre_load(P.xbn, M, bn_kind & 1, bn_on ? bn_k : 0, bn_on, P.X);

    // both weight images of this chunk -> LDS (DMA, verbatim)
    tp_dma_image<8>(P.Simg + (size_t)chunk * F, lds, F);
    tp_dma_image<8>(P.Vimg + (size_t)chunk * F, lds + F, F);

    // the previous layer's feature BatchNorm is applied to X here, as it is loaded (lazy BN:
    // X in HBM holds the pre-normalisation values); identity when xcoef is null
    // (XC: [sc_s | sc_v | sh] x (KC * 32), zero past M)
    if (bn_on) {
        const float2 c = bn_pre_coef(P.xbn, bn_pre, M, bn_kind, bn_k, blockIdx.x == 0);
        if (bn_kind == 0) { XC[bn_k] = c.x; XC[2 * KC * 32 + bn_k] = c.y; }
        else XC[KC * 32 + bn_k] = c.x;
    }
    for (int i = t; i < 3 * KC * 32; i += MP_THREADS) {
        const int part = i / (KC * 32), k = i - part * KC * 32;
        if (P.xbn.sums && k < M) continue;   // written above
        float v = 0.f;
        if (k < M) v = P.xcoef ? P.xcoef[part * M + k] : (part < 2 ? 1.f : 0.f);
        XC[i] = v;
    }

    // edge waves: thread = (edge slot of the group, channel quad cq); per-quad constants
    const int et = t - 256, cq = et & 3, ch0 = chunk * 16 + 4 * cq;
    const bool live = !gemm_wave && ch0 < M;   // M % 4 == 0: a live quad is live in all 4 lanes
    float4 ea0{}, eg0{}, et0{}, ea1{}, eg1{}, et1{}, ba{}, bg{};
    if (live) {
        auto ld4 = [&](int o) { return *reinterpret_cast<const float4*>(P.amf + o + ch0); };
        ea0 = ld4(0); eg0 = ld4(M); et0 = ld4(2 * M); ea1 = ld4(3 * M); eg1 = ld4(4 * M); et1 = ld4(5 * M);
        ba = *reinterpret_cast<const float4*>(P.bias + ch0);
        bg = *reinterpret_cast<const float4*>(P.bias + M + ch0);
    }
    // DEC hand-off counters, one per wave (the four GEMM waves and the four edge waves are not in lock
    // step with each other: a sum over the waves could reach a stage's count while one wave is still a
    // group behind -- r05: that race corrupted a group's edges about once per 100 forwards):
    // hand[p] = groups GEMM wave p has written, hand[4 + q] = groups edge wave q has read
    int* hand = reinterpret_cast<int*>(XC + 3 * KC * 32);
    if (DEC && t < 8) hand[t] = 0;
    // CHK: stage tags gtag[buf][p] = last group GEMM wave p wrote into buffer buf, etag[buf][q] = last
    // group edge wave q read from it
    int* gtag = hand + 8;
    int* etag = gtag + 4 * NBUF;
    if (CHK && t < 8 * NBUF) gtag[t] = -1;
    auto chk_fail = [&](int group, int buf, int who, int expect, int got) {
        const unsigned n = __hip_atomic_fetch_add(P.check, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (n < 8)   // the first few of a run
            printf("msg_pre hand-off mismatch: block %d wave %d group %d buffer %d: tag of wave %d is %d, expected %d\n",
               (int)blockIdx.x, wave, group, buf, who, got, expect);
    };
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // relaxed LDS poll until all four counters of a role reach `groups` (the LDS keeps each wave's
    // operations in order; the empty asm keeps the compiler from hoisting the exchange accesses above
    // it), and a no-return LDS add to the wave's own counter after its LDS traffic (inline asm: no
    // wait for the wave's global stores)
    auto dec_wait = [&](int role, int groups) {
        const int* h = hand + 4 * role;
        auto low = [&]() {
            int m = __hip_atomic_load(h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
            for (int w = 1; w < 4; ++w) {
                const int v = __hip_atomic_load(h + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                m = v < m ? v : m;
            }
            return m;
        };
        while (low() < groups) __builtin_amdgcn_s_sleep(1);
        asm volatile("" ::: "memory");
    };
    auto dec_signal = [&](int role) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) {
            const unsigned a = (unsigned)(uintptr_t)(hand + 4 * role + (wave & 3));
            asm volatile("ds_add_u32 %0, %1" ::"v"(a), "v"(1) : "memory");
        }
    };

    const float* img = lds + (plane ? F : 0);
    const int group_items = NG * G;
    unsigned long long c_mark = P.dbg ? clock64() : 0ull, c_gemm = 0ull, c_ex = 0ull, c_edge = 0ull;
    const unsigned long long c_stage = c_mark;
    auto tick = [&](unsigned long long& acc) {
        if (P.dbg) { const unsigned long long c = clock64(); acc += c - c_mark; c_mark = c; }
    };
    // edge waves: the geometry of the thread's first edge slot of the next group, prefetched
    // one stage ahead
    auto load_geo = [&](int gi, float4& g4, float& pm) {
        const int64_t e = ((int64_t)(pblk + gi * P.per_chunk) * NG) * G + (et >> 2);
        const bool ok = live && gi < my_groups && (et >> 2) < group_items && e < Ep;
        g4 = ok ? *reinterpret_cast<const float4*>(P.EG + e * 8) : float4{0.f, 0.f, 0.f, 0.f};
        pm = ok ? P.EG[e * 8 + 4] : 0.f;
    };
    float4 geo_next{};
    float pm_next = 0.f;
    load_geo(0, geo_next, pm_next);
    for (int i = 0; i <= my_groups; ++i) {
        floatx4 acc[6];
        auto write_ex = [&](int buf) {
            if constexpr (DEC)   // buffer `buf` free: the edge waves are done with group i - NBUF
                if (i >= NBUF) dec_wait(1, i - NBUF + 1);
            if constexpr (CHK != 0 && DEC) {
                if (i >= NBUF && lane == 0)
                    for (int q = 0; q < 4; ++q) {
                        const int g = __hip_atomic_load(etag + 4 * buf + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        if (g != i - NBUF) chk_fail(i, buf, 4 + q, i - NBUF, g);
                    }
            }
            float* ex = EX + buf * MP_EX + plane * 6 * MP_PART;
            float z = 0.f;   // fp16x2 range guard (tp_fused.h tp_range_flag)
#pragma unroll
            for (int j = 0; j < 6; ++j)
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    const int col = X3 ? (c16 & 3) | (((c16 >> 2) ^ qd) << 2) : c16;   // row (4 qd + jj) >> 2 = qd
                    ex[j * MP_PART + (4 * qd + jj) * MP_RS + col] = PREC == 2 ? acc[j][jj] * P.bscale : acc[j][jj];
                    if constexpr (PREC == 2) z = tp_nonfinite_fold(z, acc[j][jj]);
                }
            if constexpr (PREC == 2) tp_range_flag(P.range_flag, z);
        };
        if (gemm_wave) {
            if (i < my_groups) {
                // ---- node GEMM of group i: 16 rows x 96 columns (6 parts x 16 channels)
#pragma unroll
                for (int j = 0; j < 6; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
                if constexpr (X3) {
                    // Split-precision node GEMM, static over the KCT chunks.  Chunk kc+1's B
                    // fragments are read while the second half of chunk kc's MFMAs issues, into
                    // registers last read by chunk kc-1's MFMAs -- at least 18 MFMAs (288 cycles)
                    // earlier, so no pending MFMA's operands are refilled (msg_pre.hip history:
                    // LDS returns overwriting the operands of a pending MFMA corrupted groups).
                    using SP = SplitP<PREC>;
                    using SPT = typename SP::T;
                    constexpr int NP = SP::NP, NT = SP::NT;
                    const SPT* bimg = reinterpret_cast<const SPT*>(img) + lane;
                    SPT bx[2][6][NP], ax[2][NP];
                    auto read_b = [&](int kc, SPT (&bb)[6][NP]) {
#pragma unroll
                        for (int j = 0; j < 6; ++j)
#pragma unroll
                            for (int p3 = 0; p3 < NP; ++p3) bb[j][p3] = bimg[(j * KCT + kc) * (NP * 64) + p3 * 64];
                    };
                    read_b(0, bx[0]);
                    static_for<0, KCT>([&](auto kcc) {
                        constexpr int kc = decltype(kcc)::value;
                        // x = sc * x~ + sh (shift on the 0e plane only), split into bf16 x3
                        const float* xc = XC + (plane ? KCT * 32 : 0) + kc * 32 + 8 * qd;
                        const float4 sc0 = *reinterpret_cast<const float4*>(xc);
                        const float4 sc1 = *reinterpret_cast<const float4*>(xc + 4);
                        float4 sh0{0.f, 0.f, 0.f, 0.f}, sh1{0.f, 0.f, 0.f, 0.f};
                        if (plane == 0) {
                            sh0 = *reinterpret_cast<const float4*>(XC + 2 * KCT * 32 + kc * 32 + 8 * qd);
                            sh1 = *reinterpret_cast<const float4*>(XC + 2 * KCT * 32 + kc * 32 + 8 * qd + 4);
                        }
                        const float4 v0{fmaf(sc0.x, abuf[kc][0].x, sh0.x), fmaf(sc0.y, abuf[kc][0].y, sh0.y),
                                        fmaf(sc0.z, abuf[kc][0].z, sh0.z), fmaf(sc0.w, abuf[kc][0].w, sh0.w)};
                        const float4 v1{fmaf(sc1.x, abuf[kc][1].x, sh1.x), fmaf(sc1.y, abuf[kc][1].y, sh1.y),
                                        fmaf(sc1.z, abuf[kc][1].z, sh1.z), fmaf(sc1.w, abuf[kc][1].w, sh1.w)};
                        SP::split(v0, v1, ax[kc & 1]);
                        const SPT (&a)[NP] = ax[kc & 1];
                        const SPT (&b)[6][NP] = bx[kc & 1];
                        __builtin_amdgcn_sched_barrier(0);
                        // terms [0, NT/2): then the next chunk's B reads go out under terms [NT/2, NT)
#pragma unroll
                        for (int tt = 0; tt < NT / 2; ++tt)
#pragma unroll
                            for (int j = 0; j < 6; ++j) acc[j] = mfma16x16(a[SP::TA[tt]], b[j][SP::TB[tt]], acc[j]);
                        __builtin_amdgcn_sched_barrier(0);
                        if constexpr (kc + 1 < KCT) read_b(kc + 1, bx[(kc + 1) & 1]);
#pragma unroll
                        for (int tt = NT / 2; tt < NT; ++tt)
#pragma unroll
                            for (int j = 0; j < 6; ++j) acc[j] = mfma16x16(a[SP::TA[tt]], b[j][SP::TB[tt]], acc[j]);
                        __builtin_amdgcn_sched_barrier(0);
                    });
                    // the next group's B reads are 18+ MFMAs away; the A prefetch below only
                    // refills abuf (read by VALU, not by the MFMAs)
                }
                // B fragments double-buffered across the 32-deep K chunks: the reads of chunk
                // kc + 1 are in flight while chunk kc's 48 MFMAs issue
                float4 b[2][6][2];
                auto load_b = [&](int kc, float4 (&bb)[6][2]) {
#pragma unroll
                    for (int j = 0; j < 6; ++j) {
                        const float* bp = img + (j * KC + kc) * 512 + 4 * lane;
                        bb[j][0] = *reinterpret_cast<const float4*>(bp);
                        bb[j][1] = *reinterpret_cast<const float4*>(bp + 256);
                    }
                };
                if constexpr (!X3) load_b(0, b[0]);
#pragma unroll
                for (int kc = 0; kc < KCMAX; ++kc) {
                    if (X3 || kc >= KC) break;
                    if (!X3 && kc + 1 < KC) load_b(kc + 1, b[(kc + 1) & 1]);
                    // x = sc * x~ + sh (shift on the 0e plane only)
                    const float* xc = XC + (plane ? KC * 32 : 0) + kc * 32 + 8 * qd;
                    const float4 sc0 = *reinterpret_cast<const float4*>(xc);
                    const float4 sc1 = *reinterpret_cast<const float4*>(xc + 4);
                    float4 sh0{0.f, 0.f, 0.f, 0.f}, sh1{0.f, 0.f, 0.f, 0.f};
                    if (plane == 0) {
                        sh0 = *reinterpret_cast<const float4*>(XC + 2 * KC * 32 + kc * 32 + 8 * qd);
                        sh1 = *reinterpret_cast<const float4*>(XC + 2 * KC * 32 + kc * 32 + 8 * qd + 4);
                    }
                    const float av[8] = {fmaf(sc0.x, abuf[kc][0].x, sh0.x), fmaf(sc0.y, abuf[kc][0].y, sh0.y),
                                         fmaf(sc0.z, abuf[kc][0].z, sh0.z), fmaf(sc0.w, abuf[kc][0].w, sh0.w),
                                         fmaf(sc1.x, abuf[kc][1].x, sh1.x), fmaf(sc1.y, abuf[kc][1].y, sh1.y),
                                         fmaf(sc1.z, abuf[kc][1].z, sh1.z), fmaf(sc1.w, abuf[kc][1].w, sh1.w)};
                    {
                        const float4 (&bc)[6][2] = b[kc & 1];
#pragma unroll
                        for (int s = 0; s < 8; ++s)
#pragma unroll
                            for (int j = 0; j < 6; ++j)
                                acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], f4get(bc[j][s >> 2], s & 3),
                                                                              acc[j], 0, 0, 0);
                    }
                }
                // prefetch the next group's rows
#pragma unroll
                for (int kc = 0; kc < KCMAX; ++kc)
                    if (kc < KC) load_a(i + 1, kc, abuf[kc]);
                write_ex(i % NBUF);
                if constexpr (CHK != 0 && DEC) {   // stage tag after the data (the LDS keeps a wave's order)
                    if (lane == 0) __hip_atomic_store(gtag + 4 * (i % NBUF) + plane, i, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                if constexpr (DEC) dec_signal(0);
                tick(c_gemm);
            }
        } else if (i > 0 && live) {
            // ---- edges of group i-1
            const float4 geo_cur = geo_next;
            const float pm_cur = pm_next;
            load_geo(i, geo_next, pm_next);
            if constexpr (DEC && CHK != 2) dec_wait(0, i);   // group i - 1 written by all four GEMM waves
            if constexpr (CHK != 0 && DEC) {
                if ((t & 63) == 0)
                    for (int p = 0; p < 4; ++p) {
                        const int g = __hip_atomic_load(gtag + 4 * ((i - 1) % NBUF) + p, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_WORKGROUP);
                        if (g != i - 1) chk_fail(i - 1, (i - 1) % NBUF, p, i - 1, g);
                    }
                asm volatile("" ::: "memory");
            }
            const float* exb = EX + ((i - 1) % NBUF) * MP_EX;
            auto xv = [&](int pl, int part, int row) {
                const int q = X3 ? cq ^ ((row >> 2) & 3) : cq;
                return *reinterpret_cast<const float4*>(exb + (pl * 6 + part) * MP_PART + row * MP_RS + 4 * q);
            };
            const int64_t node0 = (int64_t)(pblk + (i - 1) * P.per_chunk) * NG;
            for (int it = et >> 2; it < group_items; it += 64) {
                const int ld = it >> lg, q = it & (G - 1);
                const int64_t dn = node0 + ld;
                if (dn >= P.V) break;
                const int64_t e = dn * G + q;
                const uint32_t os = (uint32_t)((e * 2 * M + ch0) * 4), ov = (uint32_t)((e * M + ch0) * 4);
                const uint32_t opl = (uint32_t)(Ep * M * 4);
                const int d = ld - N * tp_udiv_small(ld, invN);        // position in the system
                const int sq = P.slot ? P.slot[e] : (q < N - 1 ? (q < d ? q : q + 1) : -1);
                if (sq < 0) {   // padding slot
                    const float4 z{0.f, 0.f, 0.f, 0.f};
                    st4(rsS, os, z);
                    if (!P.no_dot) st4(rsS, os + 4 * M, z);
                    st4(rsV, ov, z); st4(rsV, ov + opl, z); st4(rsV, ov + 2 * opl, z);
                    continue;
                }
                const int sl = ld - d + sq;                              // source node, same group
                const bool first = it == (et >> 2);
                const float4 g4 = first ? geo_cur : *reinterpret_cast<const float4*>(P.EG + e * 8);
                const float pm = first ? pm_cur : P.EG[e * 8 + 4];
                const float hk[3] = {g4.x, g4.y, g4.z};
                const float dist = g4.w;
                // scalar per channel (no packed fp32: it runs beside the GEMM wave's MFMAs, where
                // v_pk_* ops cost extra issue cycles)
                float4 xd[4][6], xs[4][6];   // [plane][part] of the destination / source rows
#pragma unroll
                for (int pl = 0; pl < 4; ++pl)
#pragma unroll
                    for (int pt = 0; pt < 3; ++pt) {
                        xd[pl][pt] = xv(pl, pt, ld);
                        xs[pl][pt] = xv(pl, 3 + pt, sl);
                    }
                float o_ms[4], o_v0[4], o_v1[4], o_v2[4], o_dot[4];
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    auto X = [&](const float4& f) { return f4get(f, c); };
                    float sa = fmaf(X(ea1), pm, fmaf(X(ea0), dist, X(xd[0][0]) + X(xs[0][0]))) + X(ba);
                    float sg = fmaf(X(eg1), pm, fmaf(X(eg0), dist, X(xd[0][1]) + X(xs[0][1]))) + X(bg);
                    const float tt = fmaf(X(et1), pm, fmaf(X(et0), dist, X(xd[0][2]) + X(xs[0][2])));
                    float v[3];
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        sa = fmaf(hk[k], X(xd[1 + k][0]) + X(xs[1 + k][0]), sa);
                        sg = fmaf(hk[k], X(xd[1 + k][1]) + X(xs[1 + k][1]), sg);
                        v[k] = fmaf(hk[k], tt, X(xd[1 + k][2])) + X(xs[1 + k][2]);
                    }
                    const float gg = kC_SIGMOID * tp_sigmoid(sg);
                    o_ms[c] = kC_SILU * tp_silu(sa);
                    o_v0[c] = gg * v[0];
                    o_v1[c] = gg * v[1];
                    o_v2[c] = gg * v[2];
                    o_dot[c] = fmaf(o_v2[c], hk[2], fmaf(o_v1[c], hk[1], o_v0[c] * hk[0]));
                }
                st4(rsV, ov, float4{o_v0[0], o_v0[1], o_v0[2], o_v0[3]});
                st4(rsV, ov + opl, float4{o_v1[0], o_v1[1], o_v1[2], o_v1[3]});
                st4(rsV, ov + 2 * opl, float4{o_v2[0], o_v2[1], o_v2[2], o_v2[3]});
                st4(rsS, os, float4{o_ms[0], o_ms[1], o_ms[2], o_ms[3]});
                if (!P.no_dot) st4(rsS, os + 4 * M, float4{o_dot[0], o_dot[1], o_dot[2], o_dot[3]});
            }
            tick(c_edge);
        }
        if constexpr (DEC) {
            if constexpr (CHK != 0) {   // this edge wave is done reading group i - 1
                if (!gemm_wave && i > 0 && (t & 63) == 0) {
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    __hip_atomic_store(etag + 4 * ((i - 1) % NBUF) + (wave & 3), i - 1, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
            // (every edge wave signals, dead lanes or not)
            if (!gemm_wave && i > 0) dec_signal(1);
        } else {
            // LDS hand-off only: wait for this wave's LDS traffic, not for its global stores
            // (the empty asm after each barrier keeps the compiler from hoisting LDS accesses above it)
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        }
        tick(c_ex);
    }
    if (P.dbg && lane == 0) {
        unsigned long long* d = P.dbg + ((size_t)blockIdx.x * 8 + wave) * 4;
        d[0] = c_stage - c_start; d[1] = c_gemm; d[2] = c_ex; d[3] = c_edge;
    }
}

inline size_t msg_pre_lds_bytes(const MsgPreProb& p) {
    return ((size_t)2 * p.img_floats + mp_nbuf(p.prec) * (p.prec ? MpEx<true>::EX : MpEx<false>::EX) +
            3 * 32 * ((p.M + 31) / 32)) * 4 + 32 + 4 * 8 * 3;   // + the hand-off counters and stage tags
}

// NBX_MP_CHECK: the device word the check kernels count hand-off mismatches into (allocated once)
unsigned* mp_check_word() {
    static unsigned* w = nullptr;
    if (!w) {
        if (hipMalloc(&w, sizeof(unsigned)) != hipSuccess || hipMemset(w, 0, sizeof(unsigned)) != hipSuccess) {
            set_error("msg_pre: cannot allocate the NBX_MP_CHECK counter");
            w = nullptr;
        }
    }
    return w;
}

int msg_pre_launch(MsgPreProb& p, hipStream_t st, int num_cus) {
    if (p.V <= 0) return NBX_OK;
    if (p.M > 128 || p.NG <= 0 || (p.prec && p.M > 96)) {   // split images + exchange fit the LDS up to mul 96
        set_error("msg_pre: needs mul <= 128 and 2 <= N <= 16 (got mul %d, N %d)", p.M, p.N);
        return NBX_E_UNSUPPORTED;
    }
    if ((double)4 * p.V * p.M * 4.0 >= 2147483632.0 || (double)3 * p.V * p.G * p.M * 4.0 >= 2147483632.0 ||
        (double)2 * p.V * p.G * p.M * 4.0 >= 2147483632.0) {
        set_error("msg_pre: X / M1S / M1V span >= 2 GiB (32-bit buffer offsets)");
        return NBX_E_UNSUPPORTED;
    }
    p.chunks = (p.M + 15) / 16;
    p.img_floats = 6 * ((p.M + 31) / 32) * (p.prec == 1 ? 768 : 512);   // bf16x3 1.5x, fp16x2 1x fp32
    p.n_slabs = (int)((p.V + p.NG - 1) / p.NG);
    // one block per CU (LDS-bound); balance the group rounds over the chunk's blocks
    int per = num_cus / p.chunks;
    if (per < 1) per = 1;
    const int rounds = (p.n_slabs + per - 1) / per;
    per = (p.n_slabs + rounds - 1) / rounds;
    // XCD grouping needs per_chunk % 8 == 0 (NBX_MP_XCD=0: the plain chunk-major order, A/B only)
    static const bool xcd = !(getenv("NBX_MP_XCD") && getenv("NBX_MP_XCD")[0] == '0');
    p.xcd_group = xcd ? 1 : 0;
    if (xcd) per = (per + 7) / 8 * 8;
    p.per_chunk = per;
    const size_t lds = msg_pre_lds_bytes(p);
    if (lds > 160 * 1024) {
        set_error("msg_pre: %zu bytes of LDS (> 160 KiB)", lds);
        return NBX_E_UNSUPPORTED;
    }
    for (const void* k : {(const void*)msg_pre_kernel<0>, (const void*)msg_pre_kernel<1, 1>,
                          (const void*)msg_pre_kernel<1, 2>, (const void*)msg_pre_kernel<1, 3>,
                          (const void*)msg_pre_kernel<2, 1>, (const void*)msg_pre_kernel<2, 2>,
                          (const void*)msg_pre_kernel<2, 3>})
        NBX_LDS_160K(k);
    const int kct = (p.M + 31) / 32;
    const dim3 grid(p.chunks * p.per_chunk);
    // NBX_MP_CHECK=1 / 2: the hand-off invariant check (2: with the fault injection) on the fp16x2 path,
    // counted into a device word read by nbx_debug_msg_pre_check (diagnosis and tests only)
    static const int chk = getenv("NBX_MP_CHECK") ? atoi(getenv("NBX_MP_CHECK")) : 0;
    if (chk && p.prec == 2 && p.M % 16 == 0) {
        p.check = mp_check_word();
        if (!p.check) return NBX_E_HIP;
        for (const void* k : {(const void*)msg_pre_kernel<2, 1, 1>, (const void*)msg_pre_kernel<2, 2, 1>,
                              (const void*)msg_pre_kernel<2, 3, 1>, (const void*)msg_pre_kernel<2, 3, 2>})
            NBX_LDS_160K(k);
        if (kct == 3 && chk == 2) hipLaunchKernelGGL((msg_pre_kernel<2, 3, 2>), grid, dim3(MP_THREADS), lds, st, p);
        else if (kct == 3) hipLaunchKernelGGL((msg_pre_kernel<2, 3, 1>), grid, dim3(MP_THREADS), lds, st, p);
        else if (kct == 2) hipLaunchKernelGGL((msg_pre_kernel<2, 2, 1>), grid, dim3(MP_THREADS), lds, st, p);
        else hipLaunchKernelGGL((msg_pre_kernel<2, 1, 1>), grid, dim3(MP_THREADS), lds, st, p);
        NBX_HIP(hipGetLastError());
        return NBX_OK;
    }
    if (p.prec == 2 && kct == 3) NBX_TIMED_LAUNCH((msg_pre_kernel<2, 3>), grid, dim3(MP_THREADS), lds, st, p);
    else if (p.prec == 2 && kct == 2) NBX_TIMED_LAUNCH((msg_pre_kernel<2, 2>), grid, dim3(MP_THREADS), lds, st, p);
    else if (p.prec == 2 && kct == 1) NBX_TIMED_LAUNCH((msg_pre_kernel<2, 1>), grid, dim3(MP_THREADS), lds, st, p);
    else if (p.prec == 1 && kct == 3) NBX_TIMED_LAUNCH((msg_pre_kernel<1, 3>), grid, dim3(MP_THREADS), lds, st, p);
    else if (p.prec == 1 && kct == 1) NBX_TIMED_LAUNCH((msg_pre_kernel<1, 1>), grid, dim3(MP_THREADS), lds, st, p);
    else if (p.prec == 1 && kct == 2) NBX_TIMED_LAUNCH((msg_pre_kernel<1, 2>), grid, dim3(MP_THREADS), lds, st, p);
    else NBX_TIMED_LAUNCH(msg_pre_kernel<0>, grid, dim3(MP_THREADS), lds, st, p);
    NBX_HIP(hipGetLastError());
    return NBX_OK;
}

}  // namespace nbx

// NBX_MP_CHECK diagnosis: the number of hand-off invariant violations counted so far (0 when the check is off)
extern "C" int nbx_debug_msg_pre_check(uint32_t* mismatches, int32_t reset) {
    NBX_CHECK_ARG(mismatches != nullptr, "nbx_debug_msg_pre_check: null output");
    *mismatches = 0;
    static const int chk = getenv("NBX_MP_CHECK") ? atoi(getenv("NBX_MP_CHECK")) : 0;
    if (!chk) return NBX_OK;
    unsigned* w = nbx::mp_check_word();
    if (!w) return NBX_E_HIP;
    NBX_HIP(hipDeviceSynchronize());
    NBX_HIP(hipMemcpy(mismatches, w, sizeof(unsigned), hipMemcpyDeviceToHost));
    if (reset) NBX_HIP(hipMemset(w, 0, sizeof(unsigned)));
    return NBX_OK;
}
