// A1 — edge-index construction (utils/build_fully_connected_graph.py).
//
// Fully connected: one thread per edge, closed form of the reference's
// nonzero(~eye(N)) pattern + repeat + system offsets (lines 4-20): bit-exact.
// kNN: one thread per node, selection of the k nearest others (lines 42-80).
#include "nbx_internal.h"

namespace {

__global__ void fc_edge_index_kernel(int64_t E, int64_t N, int64_t* __restrict__ ei) {
    const int64_t per = N * (N - 1);
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = e / per;
        const int64_t r = e - b * per;
        const int64_t i = r / (N - 1);
        const int64_t jj = r - i * (N - 1);
        const int64_t j = jj < i ? jj : jj + 1;
        ei[e] = b * N + i;       // edge_index[0]: row (source)
        ei[E + e] = b * N + j;   // edge_index[1]: col (target)
    }
}

template <typename T>
__global__ void knn_edge_index_kernel(const T* __restrict__ loc, int64_t B, int N, int k, int64_t* __restrict__ ei) {
    const int64_t node = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (node >= B * N) return;
    const int64_t b = node / N;
    const int i = (int)(node - b * N);
    const T* sys = loc + b * N * 3;
    double d[64];
    const double xi = sys[3 * i], yi = sys[3 * i + 1], zi = sys[3 * i + 2];
    for (int j = 0; j < N; ++j) {
        const double dx = xi - (double)sys[3 * j], dy = yi - (double)sys[3 * j + 1], dz = zi - (double)sys[3 * j + 2];
        d[j] = sqrt(dx * dx + dy * dy + dz * dz);
    }
    const int64_t E = B * N * (int64_t)k;
    // selection: (k+1) smallest by (distance, index); the first (self) is dropped
    uint64_t taken = 0;
    for (int s = 0; s <= k; ++s) {
        int best = -1;
        for (int j = 0; j < N; ++j) {
            if ((taken >> j) & 1ull) continue;
            if (best < 0 || d[j] < d[best]) best = j;
        }
        taken |= 1ull << best;
        if (s > 0) {
            const int64_t e = node * k + (s - 1);
            ei[e] = b * N + i;
            ei[E + e] = b * N + best;
        }
    }
}

// A graph's adjacency per destination: ADJ[dst] bit s = an edge from local node s of dst's system.
// From an edge_index (utils/build_fully_connected_graph.py layout, [2][E] int64, row = source,
// col = target): err bits 1 out of range, 2 across systems, 4 self-loop, 8 duplicate edge.
__global__ void graph_adj_kernel(const int64_t* __restrict__ ei, int64_t E, int64_t V, int N,
                                 unsigned long long* __restrict__ adj, int* __restrict__ err) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = ei[e], t = ei[E + e];
        int bad = 0;
        if (s < 0 || t < 0 || s >= V || t >= V) bad = 1;
        else if (s / N != t / N) bad = 2;
        else if (s == t) bad = 4;
        if (bad) { atomicOr(err + (e & 63), bad); continue; }
        const unsigned long long bit = 1ull << (int)(s - (s / N) * N);
        if (atomicOr(adj + t, bit) & bit) atomicOr(err + (e & 63), 8);
    }
}

// kNN branch of build_graph_with_knn (build_fully_connected_graph.py:42-80) straight into the
// adjacency: node i's k nearest others by (fp64 distance, index), the first pick (self) dropped,
// exactly as nbx_knn_edge_index (above) selects them; edges i -> neighbour.
__global__ void knn_adj_kernel(const float* __restrict__ pos, int64_t V, int N, int k,
                               unsigned long long* __restrict__ adj) {
    const int64_t node = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (node >= V) return;
    const int64_t b = node / N;
    const int i = (int)(node - b * N);
    const float* sys = pos + b * N * 3;
    double d[33];
    const double xi = sys[3 * i], yi = sys[3 * i + 1], zi = sys[3 * i + 2];
    for (int j = 0; j < N; ++j) {
        const double dx = xi - (double)sys[3 * j], dy = yi - (double)sys[3 * j + 1], dz = zi - (double)sys[3 * j + 2];
        d[j] = sqrt(dx * dx + dy * dy + dz * dz);
    }
    unsigned long long taken = 0;
    for (int s = 0; s <= k; ++s) {
        int best = -1;
        for (int j = 0; j < N; ++j) {
            if ((taken >> j) & 1ull) continue;
            if (best < 0 || d[j] < d[best]) best = j;
        }
        taken |= 1ull << best;
        if (s > 0) atomicOr(adj + b * N + best, 1ull << i);
    }
}

// adjacency -> slot table (sources ascending) and in-degree; err bit 16: in-degree above G
// (only possible with self-loops, which the kNN selection yields for coincident nodes)
__global__ void graph_slots_kernel(const unsigned long long* __restrict__ adj, int64_t V, int G,
                                   int* __restrict__ slot, float* __restrict__ degv, int* __restrict__ err) {
    const int64_t node = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (node >= V) return;
    unsigned long long m = adj[node];
    int q = 0;
    while (m) {
        const int s = __ffsll((long long)m) - 1;
        m &= m - 1;
        if (q < G) slot[node * G + q] = s;
        ++q;
    }
    if (q > G) atomicOr(err + (node & 63), 16);
    degv[node] = (float)(q < G ? q : G);
    for (int r = q; r < G; ++r) slot[node * G + r] = -1;
}

}  // namespace

namespace nbx {

// General (non fully-connected) graphs as per-destination slot tables, shared by the SEGNN and
// PONITA kernels: slot[dst * G + q] = the q-th source (local index, ascending) of dst, -1 past
// its in-degree deg[dst].  adj [V], err [64] are scratch.
int graph_slots_from_edges(const int64_t* ei, int64_t E, int64_t V, int N, int G, unsigned long long* adj, int* slot,
                           float* deg, int* err, hipStream_t st) {
    NBX_CHECK_ARG(N >= 1 && N <= 64 && G >= 1 && G <= 64, "graph slots: need N <= 64");
    NBX_HIP(hipMemsetAsync(adj, 0, sizeof(unsigned long long) * V, st));
    NBX_HIP(hipMemsetAsync(err, 0, sizeof(int) * 64, st));
    if (E > 0) {
        const unsigned blocks = (unsigned)std::min<int64_t>(ceil_div(E, 256), 65536);
        hipLaunchKernelGGL(graph_adj_kernel, dim3(blocks), dim3(256), 0, st, ei, E, V, N, adj, err);
        NBX_LAUNCH_CHECK("graph_adj");
    }
    hipLaunchKernelGGL(graph_slots_kernel, dim3((unsigned)ceil_div(V, 256)), dim3(256), 0, st, adj, V, G, slot, deg,
                       err);
    NBX_LAUNCH_CHECK("graph_slots");
    int herr[64];
    NBX_HIP(hipMemcpyAsync(herr, err, sizeof(herr), hipMemcpyDeviceToHost, st));
    NBX_HIP(hipStreamSynchronize(st));
    int e = 0;
    for (int i = 0; i < 64; ++i) e |= herr[i];
    if (e) {
        set_error("unsupported edge_index (%s%s%s%s%s)", (e & 1) ? "node index out of range " : "",
                  (e & 2) ? "edge between systems " : "", (e & 4) ? "self-loop " : "",
                  (e & 8) ? "duplicate edge " : "", (e & 16) ? "in-degree above the slot count" : "");
        return NBX_E_INVAL;
    }
    return NBX_OK;
}

// kNN graph of the current positions (no synchronisation; a self-loop the selection can produce for
// coincident nodes is dropped if it overflows the slots)
int graph_slots_from_knn(const float* pos, int64_t V, int N, int G, int k, unsigned long long* adj, int* slot,
                         float* deg, int* err, hipStream_t st) {
    NBX_CHECK_ARG(N >= 2 && N <= 33 && k >= 1 && k < N, "graph slots: need 1 <= k < N <= 33");
    NBX_HIP(hipMemsetAsync(adj, 0, sizeof(unsigned long long) * V, st));
    hipLaunchKernelGGL(knn_adj_kernel, dim3((unsigned)ceil_div(V, 128)), dim3(128), 0, st, pos, V, N, k, adj);
    NBX_LAUNCH_CHECK("knn_adj");
    hipLaunchKernelGGL(graph_slots_kernel, dim3((unsigned)ceil_div(V, 256)), dim3(256), 0, st, adj, V, G, slot, deg,
                       err);
    NBX_LAUNCH_CHECK("graph_slots");
    return NBX_OK;
}

}  // namespace nbx

extern "C" int nbx_fc_edge_index(int64_t batch_size, int64_t num_nodes, int64_t* edge_index, void* stream) {
    NBX_CHECK_ARG(batch_size >= 0 && num_nodes >= 1, "nbx_fc_edge_index: bad sizes B=%lld N=%lld",
                  (long long)batch_size, (long long)num_nodes);
    const int64_t E = batch_size * num_nodes * (num_nodes - 1);
    if (E == 0) return NBX_OK;
    NBX_CHECK_ARG(edge_index != nullptr, "nbx_fc_edge_index: null output");
    const int threads = 256;
    const int64_t blocks = std::min<int64_t>(nbx::ceil_div(E, threads), 65536);
    hipLaunchKernelGGL(fc_edge_index_kernel, dim3((unsigned)blocks), dim3(threads), 0, (hipStream_t)stream, E,
                       num_nodes, edge_index);
    NBX_LAUNCH_CHECK("fc_edge_index_kernel");
    return NBX_OK;
}

extern "C" int nbx_knn_edge_index(const void* loc, int32_t dtype, int64_t batch_size, int64_t num_nodes, int64_t k,
                                  int64_t* edge_index, void* stream) {
    NBX_CHECK_ARG(k < num_nodes, "Graph cannot have more neighbors than there are nodes in simulation - 1");
    NBX_CHECK_ARG(k >= 1 && num_nodes <= 64 && batch_size >= 0, "nbx_knn_edge_index: need 1 <= k < N <= 64");
    NBX_CHECK_ARG(dtype == 0 || dtype == 1, "nbx_knn_edge_index: dtype must be 0 (fp32) or 1 (fp64)");
    const int64_t V = batch_size * num_nodes;
    if (V == 0) return NBX_OK;
    const int threads = 128;
    const unsigned blocks = (unsigned)nbx::ceil_div(V, threads);
    if (dtype == 0)
        hipLaunchKernelGGL(knn_edge_index_kernel<float>, dim3(blocks), dim3(threads), 0, (hipStream_t)stream,
                           (const float*)loc, batch_size, (int)num_nodes, (int)k, edge_index);
    else
        hipLaunchKernelGGL(knn_edge_index_kernel<double>, dim3(blocks), dim3(threads), 0, (hipStream_t)stream,
                           (const double*)loc, batch_size, (int)num_nodes, (int)k, edge_index);
    NBX_LAUNCH_CHECK("knn_edge_index_kernel");
    return NBX_OK;
}
