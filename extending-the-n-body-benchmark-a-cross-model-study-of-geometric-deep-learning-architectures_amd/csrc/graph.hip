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

}  // namespace

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
