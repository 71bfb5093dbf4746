/* ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Restatement of the fp32 2-norm the reference computes on the CPU:
 *   fl_pytorch/utils/compressors.py:272   pnorm = torch.norm(x, p=self.p)     (p = 2, x fp32 [D])
 * torch 2.10's CPU kernel for a contiguous fp32 vector (ATen ReduceOpsKernel.cpp,
 * norm_kernel_tensor_iterator_impl, the "p == 2, reduce last dim" vectorised branch) keeps ONE
 * Vectorized<float> accumulator of 8 lanes (the 256-bit kernel this build dispatches), adds
 * x[8k + l]^2 into lane l in order as a fused multiply-add, stores the 8 lanes, sums them
 * left to right into lane 0, adds the D % 8 tail elements' squares in order (fused), and takes
 * sqrtf.  Determined empirically against torch.norm in the development container (69 of 69
 * random vectors, D from 1 to 1 000 003, mixed magnitudes; tests/test_host.py) and pinned by
 * the reference's own norms at D = 25 M (tests/golden/rows.json pnorm_bits).
 * ASSUMPTION: torch's AVX2 (8-lane) norm kernel, which x86 hosts with AVX2 run — AVX512
 * hosts too, the kernel has no AVX512 registration (this container's torch reports AVX512 and
 * matches; tests/test_host.py).  A torch without AVX2 kernels is unpinned.
 * Every operation is fp32 with one rounding (fmaf): the C compiler must not contract or
 * reassociate (-ffp-contract=off, no -ffast-math).
 */
#include <math.h>
#include <stdint.h>

float orc_torch_norm2(const float* x, int64_t d) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const int64_t m = d - d % 8;
    for (int64_t k = 0; k < m; k += 8)
        for (int l = 0; l < 8; ++l) acc[l] = fmaf(x[k + l], x[k + l], acc[l]);
    float b = acc[0];
    for (int l = 1; l < 8; ++l) b = b + acc[l];
    for (int64_t k = m; k < d; ++k) b = fmaf(x[k], x[k], b);
    return sqrtf(b);
}
