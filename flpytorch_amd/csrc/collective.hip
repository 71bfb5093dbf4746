// Multi-GPU combine on a caller-owned RCCL communicator ("a multi-GPU helper that takes
// a caller-owned RCCL communicator"; §8e).  Each rank holds the exact client-order partial sum
// sum_i w_i C_i(row_i) of its client block (flc_encode_reduce with w_total = 1.0); one collective
// over xGMI combines them and every rank divides by the global weight:
//   FLC_COMBINE_ALLREDUCE  ncclAllReduce(sum) in place — bandwidth-optimal, RCCL's summation order
//   FLC_COMBINE_ORDERED    ncclAllGather into the workspace, then a fixed rank-order fold
//                          (((p_0 + p_1) + p_2) + ...) / w_total — bit-reproducible run to run and
//                          equal on every rank
//   flc_combine_blocks     G-invariant: each rank holds the exact partials of its fixed
//                          client blocks (8 blocks, split evenly over the ranks); rank r receives column
//                          slice r of every block partial (grouped ncclSend/ncclRecv: an all-to-all),
//                          folds the blocks in block order, and one ncclAllGather assembles the result
//                          — the same bits for 1, 2, 4 or 8 GPUs, a ring all-reduce's traffic
// The reference's multi-GPU scheme (threads round-robin over devices, per-client .to(device) copies
// into the master's serverGradient, thread_pool.py:59, algorithms.py:1756) has no collective.
#include <rccl/rccl.h>

#include "common.hpp"

namespace flc {

__global__ __launch_bounds__(256) void k_div_total(float* __restrict__ p, int64_t d, float wt) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < d; j += (int64_t)gridDim.x * blockDim.x)
        p[j] = p[j] / wt;
}

// out[j] = (((parts[0][j] + parts[1][j]) + ...) + parts[nr-1][j]) / wt, rows `ld` floats apart
__global__ __launch_bounds__(256) void k_fold_ranks(const float* __restrict__ parts, int nr, int64_t ld, int64_t d,
                                                    float wt, float* __restrict__ out) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < d; j += (int64_t)gridDim.x * blockDim.x) {
        float a = parts[j];
        for (int r = 1; r < nr; ++r) a = a + parts[(int64_t)r * ld + j];
        out[j] = a / wt;
    }
}

// send[q][b][j] = blocks[b][q * s + j] (0 past d): rank q's column slice of every local block
__global__ __launch_bounds__(256) void k_pack_slices(const float* __restrict__ blocks, int64_t ld, int64_t nb,
                                                     int64_t d, int64_t s, int64_t total, float* __restrict__ send) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t q = i / (nb * s), r = i - q * nb * s;
        const int64_t b = r / s, col = q * s + (r - b * s);
        send[i] = col < d ? blocks[b * ld + col] : 0.0f;
    }
}

static int64_t slice_len(int64_t d, int nr) { return ((d + nr - 1) / nr + 3) / 4 * 4; }

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
    hipLaunchKernelGGL(k_fold_ranks, dim3(grid), dim3(256), 0, st, (const float*)d_ws, nr, d, d, w_total, d_partial);
    FLC_CHECK_LAUNCH("k_fold_ranks");
    return FLC_OK;
}

extern "C" size_t flc_combine_blocks_workspace_size(void* rccl_comm, int64_t nb_local, int64_t d) {
    int nr = 0;
    if (!rccl_comm || nb_local < 1 || d < 0 || comm_ranks(rccl_comm, &nr)) return 0;
    const int64_t s = slice_len(d, nr);
    return (size_t)(2 * nr * nb_local * s + nr * s) * sizeof(float);
}

extern "C" int flc_combine_blocks(void* rccl_comm, const float* d_blocks, int64_t ld, int64_t nb_local, int64_t d,
                                  float w_total, float* d_out, void* d_ws, size_t ws_bytes, void* stream) {
    if (!rccl_comm || nb_local < 1 || d < 0 || ld < d || (d > 0 && (!d_blocks || !d_out))) {
        set_error("flc_combine_blocks: bad comm/blocks/ld/nb_local/d");
        return FLC_ERR_ARG;
    }
    if (d == 0) return FLC_OK;
    int nr = 0, rank = 0;
    if (int rc = comm_ranks(rccl_comm, &nr)) return rc;
    ncclComm_t comm = (ncclComm_t)rccl_comm;
    if (ncclCommUserRank(comm, &rank) != ncclSuccess) { set_error("flc_combine_blocks: ncclCommUserRank failed"); return FLC_ERR_ARG; }
    const int64_t s = slice_len(d, nr), per = nb_local * s;
    const size_t need = (size_t)(2 * nr * per + nr * s) * sizeof(float);
    if (!d_ws || ws_bytes < need) { set_error("flc_combine_blocks: needs %zu workspace bytes", need); return FLC_ERR_WORKSPACE; }
    hipStream_t st = (hipStream_t)stream;
    float* send = (float*)d_ws;
    float* recv = send + nr * per;
    float* gath = recv + nr * per;
    const int64_t total = nr * per;
    hipLaunchKernelGGL(k_pack_slices, dim3((int)std::min<int64_t>((total + 255) / 256, 16384)), dim3(256), 0, st,
                       d_blocks, ld, nb_local, d, s, total, send);
    FLC_CHECK_LAUNCH("k_pack_slices");
    // the all-to-all: peer q gets my blocks' slice q, I get every peer's blocks of slice `rank`
    // (rank-major = block order, since each rank owns a contiguous run of blocks)
    bool ok = ncclGroupStart() == ncclSuccess;
    for (int q = 0; q < nr && ok; ++q) {
        ok = ncclSend(send + q * per, (size_t)per, ncclFloat32, q, comm, st) == ncclSuccess &&
             ncclRecv(recv + q * per, (size_t)per, ncclFloat32, q, comm, st) == ncclSuccess;
    }
    ok = (ncclGroupEnd() == ncclSuccess) && ok;
    if (!ok) { set_error("flc_combine_blocks: grouped ncclSend/ncclRecv failed"); return FLC_ERR_HIP; }
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((s + 255) / 256, 8192));
    hipLaunchKernelGGL(k_fold_ranks, dim3(grid), dim3(256), 0, st, (const float*)recv, (int)(nr * nb_local), s, s,
                       w_total, gath + rank * s);
    FLC_CHECK_LAUNCH("k_fold_ranks");
    if (ncclAllGather(gath + rank * s, gath, (size_t)s, ncclFloat32, comm, st) != ncclSuccess) {
        set_error("flc_combine_blocks: ncclAllGather failed");
        return FLC_ERR_HIP;
    }
    if (hipMemcpyAsync(d_out, gath, (size_t)d * sizeof(float), hipMemcpyDeviceToDevice, st) != hipSuccess) {
        set_error("flc_combine_blocks: hipMemcpyAsync failed");
        return FLC_ERR_HIP;
    }
    return FLC_OK;
}
