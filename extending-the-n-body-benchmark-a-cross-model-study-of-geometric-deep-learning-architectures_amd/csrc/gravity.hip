// A20-A22 — GravitySim softened-gravity leapfrog (datasets/nbody/dataset/synthetic_sim.py:305-420), fp64.
//
// Layout: one thread per body, the systems per workgroup (<= 1024 threads) that waste the fewest
// lanes (launch_geometry: N = 100 -> 10 systems, 1000 of 1024 lanes).  The current positions of the
// workgroup's systems live in LDS; the whole T-step KDK loop runs inside the
// kernel, so HBM only sees the initial state, the sampled frames and the final
// state.  Per step each body does N softened interactions (FP64 VALU bound).
#include "nbx_internal.h"

namespace {

// r^-1/2 for r2 > 0: the hardware v_rsq_f64 estimate refined by one Newton step,
// y1 = y0 + y0/2 (1 - r2 y0^2) (4 fp64 ops; the estimate's relative error is squared: the
// accelerations stay within 1e-14 relative of the reference, tests/test_gpu_native.py
// test_gravity_acceleration, i.e. tens of ulp rather than OCML's 1).  OCML's rsqrt adds special-case classification and a second correction: about 12 ops,
// 40 % of the pair interaction's instructions.
__device__ inline double rsqrt_nr(double r2) {
    const double y0 = __builtin_amdgcn_rsq(r2);
    const double e = fma(-r2 * y0, y0, 1.0);
    return fma(0.5 * y0, e, y0);
}

// a_i = G * sum_j ((x_j - x_i) * r^-3) * m_j, r^2 = |x_j - x_i|^2 + eps^2 (synthetic_sim.py:318-340).
// Bodies sit in LDS as (x, y, z, m) double4 (two broadcast ds_read_b128 per partner);
// r^-3 = rsqrt(r^2)^3 instead of a sqrt + divide (the reference's pow(r^2, -1.5) is itself
// ulp-different from both).
template <bool SOFT>
__device__ inline void accel_sum(const double4* __restrict__ sp, int N, double xi, double yi, double zi, double soft2,
                                 double& sx, double& sy, double& sz) {
#pragma unroll 4
    for (int j = 0; j < N; ++j) {
        const double4 p = sp[j];
        const double dx = p.x - xi, dy = p.y - yi, dz = p.z - zi;
        const double r2 = fma(dz, dz, fma(dy, dy, fma(dx, dx, soft2)));   // 3 fp64 ops
        const double ri = rsqrt_nr(r2);
        // softened (eps > 0): r2 > 0 for every pair, the self term is 0 * finite; unsoftened: the
        // self term (r2 = 0) is skipped
        const double w = SOFT ? (ri * ri * ri) * p.w : (r2 > 0.0 ? (ri * ri * ri) * p.w : 0.0);
        sx += dx * w;
        sy += dy * w;
        sz += dz * w;
    }
}

__device__ inline void accel_from_lds(const double4* __restrict__ sp, int N, double xi, double yi, double zi,
                                      double G, double soft2, double& ax, double& ay, double& az) {
    double sx = 0.0, sy = 0.0, sz = 0.0;
    if (soft2 > 0.0)
        accel_sum<true>(sp, N, xi, yi, zi, soft2, sx, sy, sz);
    else
        accel_sum<false>(sp, N, xi, yi, zi, soft2, sx, sy, sz);
    ax = G * sx;
    ay = G * sy;
    az = G * sz;
}

__global__ void gravity_accel_kernel(const double* __restrict__ pos, const double* __restrict__ mass, int64_t S, int N,
                                     int spb, double G, double soft2, double* __restrict__ acc) {
    extern __shared__ double4 lds4[];   // [spb][N] (x, y, z, m)
    const int local = threadIdx.x / N, i = threadIdx.x % N;
    const int64_t s = (int64_t)blockIdx.x * spb + local;
    const bool live = local < spb && s < S;
    double x = 0, y = 0, z = 0;
    if (live) {
        x = pos[(s * N + i) * 3 + 0];
        y = pos[(s * N + i) * 3 + 1];
        z = pos[(s * N + i) * 3 + 2];
        lds4[local * N + i] = make_double4(x, y, z, mass[s * N + i]);
    }
    __syncthreads();
    if (!live) return;
    double ax, ay, az;
    accel_from_lds(lds4 + local * N, N, x, y, z, G, soft2, ax, ay, az);
    acc[(s * N + i) * 3 + 0] = ax;
    acc[(s * N + i) * 3 + 1] = ay;
    acc[(s * N + i) * 3 + 2] = az;
}

// OCC: minimum resident 1024-thread workgroups per CU the register allocation must allow (2: <= 64
// VGPRs, 8 waves per SIMD to hide the rsq / LDS latency of the pair loop; 1: the compiler's choice)
template <int OCC>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(4 * OCC))) void gravity_sample_kernel(double* __restrict__ pos, double* __restrict__ vel,
                                      const double* __restrict__ mass, int64_t S, int N, int spb, int64_t T,
                                      int64_t freq, double dt, double G, double soft2, double* __restrict__ pos_save,
                                      double* __restrict__ vel_save, double* __restrict__ force_save) {
    extern __shared__ double4 lds4[];   // [spb][N] (x, y, z, m)
    const int local = threadIdx.x / N, i = threadIdx.x % N;
    const int64_t s = (int64_t)blockIdx.x * spb + local;
    const bool live = local < spb && s < S;
    const int64_t Ts = T / freq;
    double x = 0, y = 0, z = 0, vx = 0, vy = 0, vz = 0, m = 0;
    double4* sp = lds4 + (live ? local * N : 0);
    if (live) {
        x = pos[(s * N + i) * 3 + 0];
        y = pos[(s * N + i) * 3 + 1];
        z = pos[(s * N + i) * 3 + 2];
        vx = vel[(s * N + i) * 3 + 0];
        vy = vel[(s * N + i) * 3 + 1];
        vz = vel[(s * N + i) * 3 + 2];
        m = mass[s * N + i];
        sp[i] = make_double4(x, y, z, m);
    }
    __syncthreads();
    double ax = 0, ay = 0, az = 0;
    if (live) accel_from_lds(sp, N, x, y, z, G, soft2, ax, ay, az);
    const double hdt = dt / 2.0;
    int64_t c = 0;
    for (int64_t t = 0; t < T; ++t) {
        if (live && t % freq == 0) {
            const int64_t o = ((s * Ts + c) * N + i) * 3;
            pos_save[o] = x; pos_save[o + 1] = y; pos_save[o + 2] = z;
            vel_save[o] = vx; vel_save[o + 1] = vy; vel_save[o + 2] = vz;
            force_save[o] = ax * m; force_save[o + 1] = ay * m; force_save[o + 2] = az * m;
            ++c;
        }
        // (1/2) kick, drift
        vx += ax * hdt; vy += ay * hdt; vz += az * hdt;
        x += vx * dt; y += vy * dt; z += vz * dt;
        __syncthreads();  // everyone finished reading the previous positions
        if (live) sp[i] = make_double4(x, y, z, m);
        __syncthreads();
        if (live) accel_from_lds(sp, N, x, y, z, G, soft2, ax, ay, az);
        // (1/2) kick
        vx += ax * hdt; vy += ay * hdt; vz += az * hdt;
    }
    if (live) {
        pos[(s * N + i) * 3 + 0] = x; pos[(s * N + i) * 3 + 1] = y; pos[(s * N + i) * 3 + 2] = z;
        vel[(s * N + i) * 3 + 0] = vx; vel[(s * N + i) * 3 + 1] = vy; vel[(s * N + i) * 3 + 2] = vz;
    }
}

// Trainer._compute_nbody_energies (trainer.py:888-927) per (system, frame):
// kinetic = 0.5 sum v^2 (unit masses), potential = -G sum_{i<j} 1/sqrt(|x_i - x_j|^2 + eps^2)
// (a zero distance with eps = 0 contributes 0, like the reference's inv_r > 0 mask).
__global__ void nbody_energy_kernel(const double* __restrict__ loc, const double* __restrict__ vel, int64_t F, int N,
                                    double G, double soft2, double* __restrict__ kin, double* __restrict__ pot) {
    const int64_t f = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (f >= F) return;
    const double* x = loc + f * N * 3;
    const double* v = vel + f * N * 3;
    double k = 0.0;
    for (int i = 0; i < 3 * N; ++i) k += v[i] * v[i];
    double s = 0.0;
    for (int i = 0; i < N; ++i)
        for (int j = i + 1; j < N; ++j) {
            const double dx = x[3 * j] - x[3 * i], dy = x[3 * j + 1] - x[3 * i + 1], dz = x[3 * j + 2] - x[3 * i + 2];
            const double r = sqrt(dx * dx + dy * dy + dz * dz + soft2);
            s += r > 0.0 ? 1.0 / r : 0.0;
        }
    kin[f] = 0.5 * k;
    pot[f] = -G * s;
}

// out[t] = mean over systems b of x[b, t]
__global__ void batch_mean_kernel(const double* __restrict__ x, int64_t B, int64_t T, double* __restrict__ out) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t >= T) return;
    double s = 0.0;
    for (int64_t b = 0; b < B; ++b) s += x[b * T + t];
    out[t] = s / (double)B;
}

// Systems per workgroup: the count (up to 1024 threads) that wastes the fewest lanes of
// the last wave, smallest on ties; e.g. N = 100 -> 10 systems = 1000 of 1024 lanes busy.
void launch_geometry(int64_t N, int& spb, int& threads) {
    if (N > 1024) N = 1024;
    int best = 1;
    double best_u = 0.0;
    for (int s = 1; s * N <= 1024; ++s) {
        const int th = ((s * (int)N + 63) / 64) * 64;
        const double u = (double)(s * N) / th;
        if (u > best_u + 1e-9) {
            best_u = u;
            best = s;
        }
    }
    spb = best;
    threads = ((spb * (int)N + 63) / 64) * 64;
}

}  // namespace

extern "C" int nbx_gravity_acceleration(const double* pos, const double* mass, int64_t S, int64_t N, double G,
                                        double softening, double* acc, void* stream) {
    NBX_CHECK_ARG(S >= 0 && N >= 1 && N <= 1024, "nbx_gravity_acceleration: need 1 <= N <= 1024");
    if (S == 0) return NBX_OK;
    int spb, threads;
    launch_geometry(N, spb, threads);
    const size_t lds = sizeof(double4) * spb * N;
    hipLaunchKernelGGL(gravity_accel_kernel, dim3((unsigned)nbx::ceil_div(S, spb)), dim3(threads), lds,
                       (hipStream_t)stream, pos, mass, S, (int)N, spb, G, softening * softening, acc);
    NBX_LAUNCH_CHECK("gravity_accel_kernel");
    return NBX_OK;
}

extern "C" int nbx_gravity_sample(double* pos, double* vel, const double* mass, int64_t S, int64_t N, int64_t T,
                                  int64_t sample_freq, double dt, double G, double softening, double* pos_save,
                                  double* vel_save, double* force_save, void* stream) {
    NBX_CHECK_ARG(S >= 0 && N >= 1 && N <= 1024, "nbx_gravity_sample: need 1 <= N <= 1024");
    NBX_CHECK_ARG(sample_freq > 0 && T >= 0 && T % sample_freq == 0, "nbx_gravity_sample: T %% sample_freq != 0");
    if (S == 0) return NBX_OK;
    int spb, threads;
    launch_geometry(N, spb, threads);
    const size_t lds = sizeof(double4) * spb * N;
    // NBX_GRAV_OCC=1: the compiler's register allocation (one workgroup per CU at N = 100), A/B
    static const bool occ2 = !(getenv("NBX_GRAV_OCC") && getenv("NBX_GRAV_OCC")[0] == '1');
    if (occ2)
        hipLaunchKernelGGL(gravity_sample_kernel<2>, dim3((unsigned)nbx::ceil_div(S, spb)), dim3(threads), lds,
                           (hipStream_t)stream, pos, vel, mass, S, (int)N, spb, T, sample_freq, dt, G,
                           softening * softening, pos_save, vel_save, force_save);
    else
        hipLaunchKernelGGL(gravity_sample_kernel<1>, dim3((unsigned)nbx::ceil_div(S, spb)), dim3(threads), lds,
                           (hipStream_t)stream, pos, vel, mass, S, (int)N, spb, T, sample_freq, dt, G,
                           softening * softening, pos_save, vel_save, force_save);
    NBX_LAUNCH_CHECK("gravity_sample_kernel");
    return NBX_OK;
}

extern "C" int nbx_nbody_energies(const double* loc, const double* vel, int64_t B, int64_t T, int64_t N, double G,
                                  double softening, double* kinetic, double* potential, double* mean_kinetic,
                                  double* mean_potential, void* stream) {
    NBX_CHECK_ARG(B >= 0 && T >= 0 && N >= 1 && N <= 4096, "nbx_nbody_energies: bad shape");
    NBX_CHECK_ARG(kinetic && potential, "nbx_nbody_energies: kinetic/potential outputs required");
    const int64_t F = B * T;
    if (F == 0) return NBX_OK;
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(nbody_energy_kernel, dim3((unsigned)nbx::ceil_div(F, 256)), dim3(256), 0, st, loc, vel, F,
                       (int)N, G, softening * softening, kinetic, potential);
    if (mean_kinetic)
        hipLaunchKernelGGL(batch_mean_kernel, dim3((unsigned)nbx::ceil_div(T, 256)), dim3(256), 0, st, kinetic, B, T,
                           mean_kinetic);
    if (mean_potential)
        hipLaunchKernelGGL(batch_mean_kernel, dim3((unsigned)nbx::ceil_div(T, 256)), dim3(256), 0, st, potential, B,
                           T, mean_potential);
    NBX_LAUNCH_CHECK("nbody_energy_kernel");
    return NBX_OK;
}
