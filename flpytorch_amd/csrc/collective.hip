// Multi-GPU combine on a caller-owned RCCL communicator ("a multi-GPU helper that takes
// a caller-owned RCCL communicator"; §8e).  Each rank holds the exact client-order partial sum
// sum_i w_i C_i(row_i) of its client block (flc_encode_reduce with w_total = 1.0); one collective
// over xGMI combines them and every rank divides by the global weight:
//   FLC_COMBINE_ALLREDUCE  ncclAllReduce(sum) in place — bandwidth-optimal, RCCL's summation order
//   FLC_COMBINE_ORDERED    ncclAllGather into the workspace, then a fixed rank-order fold
//                          (((p_0 + p_1) + p_2) + ...) / w_total — bit-reproducible run to run and
//                          equal on every rank
// The reference's multi-GPU scheme (threads round-robin over devices, per-client .to(device) copies
// into the master's serverGradient, thread_pool.py:59, algorithms.py:1756) has no collective.
#include <rccl/rccl.h>

#include "common.hpp"

namespace flc {

__global__ __launch_bounds__(256) void k_div_total(float* __restrict__ p, int64_t d, float wt) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < d; j += (int64_t)gridDim.x * blockDim.x)
        p[j] = p[j] / wt;
}

__global__ __launch_bounds__(256) void k_fold_ranks(const float* __restrict__ parts, int nr, int64_t d, float wt,
                                                    float* __restrict__ out) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < d; j += (int64_t)gridDim.x * blockDim.x) {
        float a = parts[j];
        for (int r = 1; r < nr; ++r) a = a + parts[(int64_t)r * d + j];
        out[j] = a / wt;
    }
}

static int comm_ranks(void* comm, int* nr) {
    if (ncclCommCount((ncclComm_t)comm, nr) != ncclSuccess || *nr < 1) {
        set_error("flc_combine: ncclCommCount failed (not an RCCL communicator?)");
        return FLC_ERR_ARG;
    }
    return FLC_OK;
}

}  // namespace flc

using namespace flc;

extern "C" size_t flc_combine_workspace_size(void* rccl_comm, int64_t d, int mode) {
    if (mode != FLC_COMBINE_ORDERED || !rccl_comm || d < 0) return 0;
    int nr = 0;
    if (comm_ranks(rccl_comm, &nr)) return 0;
    return (size_t)nr * (size_t)d * sizeof(float);
}

extern "C" int flc_combine_partials(void* rccl_comm, float* d_partial, int64_t d, float w_total, int mode, void* d_ws,
                                    size_t ws_bytes, void* stream) {
    if (!rccl_comm || d < 0 || (d > 0 && !d_partial)) { set_error("flc_combine_partials: bad comm/partial/d"); return FLC_ERR_ARG; }
    if (mode != FLC_COMBINE_ALLREDUCE && mode != FLC_COMBINE_ORDERED) { set_error("flc_combine_partials: mode %d", mode); return FLC_ERR_ARG; }
    if (d == 0) return FLC_OK;
    hipStream_t st = (hipStream_t)stream;
    ncclComm_t comm = (ncclComm_t)rccl_comm;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((d + 255) / 256, 8192));
    if (mode == FLC_COMBINE_ALLREDUCE) {
        if (ncclAllReduce(d_partial, d_partial, (size_t)d, ncclFloat32, ncclSum, comm, st) != ncclSuccess) {
            set_error("flc_combine_partials: ncclAllReduce failed");
            return FLC_ERR_HIP;
        }
        hipLaunchKernelGGL(k_div_total, dim3(grid), dim3(256), 0, st, d_partial, d, w_total);
        FLC_CHECK_LAUNCH("k_div_total");
        return FLC_OK;
    }
    int nr = 0;
    if (int rc = comm_ranks(rccl_comm, &nr)) return rc;
    if (!d_ws || ws_bytes < (size_t)nr * (size_t)d * sizeof(float)) {
        set_error("flc_combine_partials: ordered mode needs %zu workspace bytes", (size_t)nr * (size_t)d * sizeof(float));
        return FLC_ERR_WORKSPACE;
    }
    if (ncclAllGather(d_partial, d_ws, (size_t)d, ncclFloat32, comm, st) != ncclSuccess) {
        set_error("flc_combine_partials: ncclAllGather failed");
        return FLC_ERR_HIP;
    }
    hipLaunchKernelGGL(k_fold_ranks, dim3(grid), dim3(256), 0, st, (const float*)d_ws, nr, d, w_total, d_partial);
    FLC_CHECK_LAUNCH("k_fold_ranks");
    return FLC_OK;
}
