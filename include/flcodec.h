/*
 * flcodec — MI355X (gfx950) gradient codecs + N-way reduction: the C ABI.
 *
 * The drop-in boundary for FL_PyTorch's simulated-uplink hot path.  The reference is pure
 * Python; the Python layer in flpytorch_amd/aggregation binds these entry points with ctypes
 * (INTEGRATION.md shows the binding) and keeps the reference's object protocol on top:
 *   - Compressor.generateCompressPattern / compressVector   fl_pytorch/utils/compressors.py:196-371
 *   - <Algorithm>.serverGradient                           fl_pytorch/utils/algorithms.py:1748-1770,
 *                                                          1810-1832 (+ the identical cores listed
 *                                                          in SURVEY.md §8a row a14)
 *
 * Conventions
 *   - every pointer named d_* is DEVICE memory (caller-owned; the library never frees it);
 *     h_* is host memory.  fp32 data only (other dtypes: FLC_ERR_DTYPE).
 *   - every compute call is asynchronous on `stream` (a hipStream_t, passed as void*), never
 *     synchronises the device, never allocates: scratch comes from a caller workspace sized by
 *     the matching *_workspace_size query.  Calls are reentrant across host threads that use
 *     distinct streams and distinct workspaces.
 *   - return 0 (FLC_OK) or an flc_status; flc_last_error_string() gives the detail for the
 *     calling thread.
 */
#ifndef FLCODEC_H
#define FLCODEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    FLC_OK = 0,
    FLC_ERR_ARG = 1,        /* bad size / null pointer / misaligned where alignment is required */
    FLC_ERR_DTYPE = 2,      /* not fp32 */
    FLC_ERR_HIP = 3,        /* a HIP runtime call failed (launch, memset) */
    FLC_ERR_WORKSPACE = 4,  /* workspace smaller than *_workspace_size() */
    FLC_ERR_UNSUPPORTED = 5 /* codec / mode not supported (e.g. a p-norm other than 1, 2, inf) */
} flc_status;

/* Codec ids = the reference's CompressorType values (compressors.py:11-19). */
typedef enum {
    FLC_IDENT = 1,
    FLC_LAZY = 2,
    FLC_RANDK = 3,
    FLC_NATURAL = 4,
    FLC_STD_DITHERING = 5,
    FLC_NAT_DITHERING = 6,
    FLC_TOPK = 7,
    FLC_RANK_K = 8          /* k = K; rank-K truncated SVD of the A x B view (compressors.py:336-364):
                               rocSOLVER / rocBLAS, parity to a stated tolerance */
} flc_codec;

/* p-norm used by the dithering codecs (Compressor.p, compressors.py:91, 123). */
#define FLC_NORM_L1 1
#define FLC_NORM_L2 2
#define FLC_NORM_LINF 0

/* Execution hints (flc_codec_params.flags).  They choose HOW a result is computed, never WHAT:
 * every combination gives the same bits.  0 = the library's choice.
 *   bits 0-1  standard dithering with p = 2: FLC_PATH_SPARSE (one-read candidate filter + exact
 *             fold) or FLC_PATH_DENSE (norm pass, then encode pass); flc_encode of one row takes
 *             the sparse pass only when FLC_PATH_SPARSE is set
 *   bits 8-15 fused encode+reduce (QSGD sparse path, TopK): number of row groups whose tails are
 *             pipelined under the next group's streaming pass (FLC_ROW_GROUPS(g), g in 1..255) */
#define FLC_PATH_AUTO 0
#define FLC_PATH_SPARSE 1
#define FLC_PATH_DENSE 2
#define FLC_PATH_MASK 3
#define FLC_ROW_GROUPS(g) (((g) & 0xFF) << 8)

/* Codec configuration — the constants Compressor.make* sets (compressors.py:64-178). */
typedef struct {
    int32_t codec;          /* flc_codec */
    int32_t s;              /* dithering: number of level intervals (levels has s+1 entries) */
    int32_t norm;           /* dithering: FLC_NORM_* */
    int32_t flags;          /* execution hints (FLC_PATH_*, FLC_ROW_GROUPS), 0 = library default */
    int64_t k;              /* randk / topk: K */
    float lazy_p;           /* lazy: P */
    float randk_scale;      /* randk: (float)(D / K) as the reference's fp32 scalar multiply */
    const float* d_levels;  /* dithering: s+1 fp32 levels (Compressor.levelsValues) on device */
    uint64_t seed;          /* device-RNG mode: experiment key of the counter-based generator */
    int32_t tie;            /* topk: which of the entries tied at the K-th magnitude are kept when
                               fewer places are left than ties (compressors.py:332 leaves it to
                               torch.topk): FLC_TIE_LOWEST (0, the lowest indices: torch.topk's CPU
                               order on the reference's rows, the oracle's rule) or FLC_TIE_HIGHEST.
                               A result, not a hint: the two rules give different sets on tied rows. */
} flc_codec_params;

#define FLC_TIE_LOWEST 0
#define FLC_TIE_HIGHEST 1

/* Patterns: where the randomness of one call comes from (generateCompressPattern, 196-216).
 * Compat mode reproduces the reference's numpy stream bit for bit (host-drawn, uploaded);
 * device mode draws from a counter-based generator keyed by (seed, client id, element). */
typedef struct {
    const int64_t* d_randk_idx; /* randk compat: [n][k] int64 indices (numpy choice(D,K)) or NULL */
    const double* d_uniforms;   /* natural / dithering compat: [n][d] float64 (numpy rand(D)) or NULL */
    const double* d_lazy_u;     /* lazy: [n] float64 draws (numpy random()) on device — required */
    int64_t client0;            /* device mode: id of row 0 (row r is client client0 + r) */
    int64_t uniforms_ld;        /* leading dimension of d_uniforms (elements); 0 = d */
    int64_t idx_ld;             /* leading dimension of d_randk_idx (elements); 0 = k */
    const uint32_t* d_randk_counts; /* randk device mode: the rows' chunk counts [ceil(d/4096)][n]
                                   * from flc_device_randk_counts with the same seed, client0, n, d,
                                   * k (e.g. computed on another stream, beside other work), or
                                   * NULL: computed inside the call */
} flc_pattern;

/* ----------------------------------------------------------------------------------------
 * Library info / errors
 * -------------------------------------------------------------------------------------- */
int flc_version(void);                    /* ABI version (major*100 + minor) */
/* Build provenance: the first 16 hex digits of sha256 over the library's sources (csrc: .hip,
 * .hpp and .cpp files in name order, then csrc/Makefile and this header), fixed at build time; "+x" is
 * appended when extra compile flags (XFLAGS) were given.  flpytorch_amd._lib.source_hash()
 * computes the same digest from a tree, so a stale .so is detected before it is measured. */
const char* flc_build_id(void);
const char* flc_last_error_string(void);  /* thread-local detail of the last failure */

/* ----------------------------------------------------------------------------------------
 * N-way reduction — the serverGradient core (algorithms.py:1753-1768).
 *
 *   mode FLC_REDUCE_REL_X : out = (sum_i w_i * (x - row_i)) / w_total      (client models in)
 *   mode FLC_REDUCE_PLAIN : out = (sum_i w_i * row_i) / w_total            (client updates in)
 *
 * Summed per element strictly in row order with fp32 rounding after every operation, i.e.
 * bit-identical to the reference's sequential loop (gs = w0*g0; gs += wi*gi; gs / w_total).
 * d_w: n fp32 weights (the reference's python-float weights as fp32), or NULL for all 1.0.
 * w_total: the python-float sum of the weights, as the fp32 divisor.
 * Rows come either as a device array of n row pointers (flc_reduce_rows; every row pointer,
 * d_x and d_out 16-byte aligned) or as one strided matrix (flc_reduce_matrix, row i at
 * d_rows + i*ld; any alignment, the vector path needs 16-byte rows and ld % 4 == 0).
 * -------------------------------------------------------------------------------------- */
#define FLC_REDUCE_PLAIN 0
#define FLC_REDUCE_REL_X 1
int flc_reduce_rows(const float* const* d_row_ptrs, int64_t n, int64_t d, const float* d_x,
                    const float* d_w, float w_total, int mode, float* d_out, void* stream);
int flc_reduce_matrix(const float* d_rows, int64_t ld, int64_t n, int64_t d, const float* d_x,
                      const float* d_w, float w_total, int mode, float* d_out, void* stream);

/* ----------------------------------------------------------------------------------------
 * Single-vector encode — Compressor.compressVector(x) (compressors.py:218-371): dense fp32
 * output `d_out[d]` (zeros where the codec sends nothing).  `row` selects pattern row 0.
 *   d_pnorm_in : dithering only — device fp32 norm to use instead of computing one (the norm
 *                the server receives on the wire), or NULL
 *   d_pnorm_out: dithering only — device fp32 where the norm used is written, or NULL
 * -------------------------------------------------------------------------------------- */
size_t flc_encode_workspace_size(const flc_codec_params* prm, int64_t d);
int flc_encode(const flc_codec_params* prm, const flc_pattern* pat, const float* d_x, int64_t d,
               const float* d_pnorm_in, float* d_pnorm_out, float* d_out, void* d_ws,
               size_t ws_bytes, void* stream);

/* Rows per flc_encode_reduce / flc_unpack_reduce call (larger rounds: fold the row blocks as
 * partials with w_total = 1 and combine them, as the multi-GPU path does). */
#define FLC_MAX_ROWS 65535

/* ----------------------------------------------------------------------------------------
 * Fused batch encode + reduce — the simulated uplink of one round in one call:
 *     out = (sum_i w_i * C_i(row_i)) / w_total
 * with C_i the codec applied to client row i under its own pattern, summed in row order
 * (bit-identical to reducing the dense compressVector outputs sequentially).  Rows are the
 * strided matrix d_rows (row i at d_rows + i*ld, ld % 4 == 0 and 16-byte alignment for the
 * vector path) — or, with d_rows == NULL, the device pointer array d_row_ptrs (every row
 * 16-byte aligned).
 * d_pnorms_out: optional [n] fp32 norms used (dithering).
 * -------------------------------------------------------------------------------------- */
size_t flc_encode_reduce_workspace_size(const flc_codec_params* prm, int64_t n, int64_t d);
int flc_encode_reduce(const flc_codec_params* prm, const flc_pattern* pat, const float* d_rows,
                      int64_t ld, const float* const* d_row_ptrs, int64_t n, int64_t d,
                      const float* d_w, float w_total, float* d_pnorms_out, float* d_out,
                      void* d_ws, size_t ws_bytes, void* stream);

/* ----------------------------------------------------------------------------------------
 * Shift codecs — the client-side update of the compressed algorithms,
 * one client row, with e = C(a - b) never stored for the elementwise codecs:
 *     d_msg       = d_base + e * msg_scale        (e * msg_scale when d_base == NULL)
 *     d_shift_out = d_shift_in + shift_alpha * e
 * each op rounded separately in fp32, like the torch expressions it replaces:
 *   DIANA  m = C(g - h); h = h + alpha * m              algorithms.py:1383-1391
 *          -> a=g, b=h, msg_scale=1, msg=m, shift_in=h, shift_out=h', alpha=(float)alpha
 *   EF21   g_next = g_prev + C(g - g_prev) * mult      algorithms.py:1506-1517
 *          -> a=g, b=g_prev, base=g_prev, msg_scale=(float)mult, msg=g_next
 *   MARINA g_next = g_prev + C(g - g_prev_x)           algorithms.py:537, 691
 *   FRECON / COFIG u = C(g - h); h = h + alpha * u     algorithms.py:1104-1110, 1265-1269
 * C follows prm / pat exactly as in flc_encode (same patterns, same draws).  d_msg or
 * d_shift_out may be NULL (not written), not both; outputs may alias any input (every element
 * is read before it is written, by the same thread).  d_pnorm_out: optional norm of a - b
 * (dithering).
 * -------------------------------------------------------------------------------------- */
size_t flc_encode_shift_workspace_size(const flc_codec_params* prm, int64_t d);
int flc_encode_shift(const flc_codec_params* prm, const flc_pattern* pat, const float* d_a,
                     const float* d_b, int64_t d, float msg_scale, const float* d_base, float* d_msg,
                     float shift_alpha, const float* d_shift_in, float* d_shift_out,
                     float* d_pnorm_out, void* d_ws, size_t ws_bytes, void* stream);

/* ----------------------------------------------------------------------------------------
 * Wire format: the message a client sends, and the server's decode +
 * reduce straight from the N messages.  The reference counts these bits
 * (last_need_to_send_advance, compressors.py:223-224, 367-368) but moves the dense decoded
 * tensor (comm_socket.py:16-82 pickles it).  One row's payload = 16-B header
 * {u32 format, u32 count, f32 norm, u32 bad} + body, padded to 16 B:
 *   1 F32    ident, lazy, natural dithering                f32[d]
 *   2 Q8     std dithering / qsgd / terngrad, s <= 127     u8[d]: bit 7 sign, bits 0-6 level index
 *   3 Q16    std dithering, s > 127                        u16[d]: bit 15 sign, bits 0-14 level index
 *   4 NAT16  natural                                       u16[d]: bit 15 sign; 0 zero, 0x7FFE inf,
 *                                                          0x7FFF NaN, else k + 16384 for 2^k
 *   5 SPARSE randk, topk                                   u32 idx[K] then f32 val[K] (count used,
 *                                                          ascending idx, the elements not +0)
 *   6 RANKK  rank_k                                        the rank-K' expansion, f32: U'_K (B x K')
 *                                                          then (S V'^T)_K' (K' x A), each 16-B
 *                                                          padded — K' (A + B) values, count = K'
 *                                                          (decoded by the encode's own GEMM)
 * Level code 0 is +0; otherwise value = (levels[idx] * sign) * norm (compressors.py:294-296).
 * flc_unpack(flc_pack(x)) == flc_encode(x) bit for bit; flc_unpack_reduce(payloads) ==
 * flc_encode_reduce(rows).  flc_pack runs the encode (same patterns and draws as flc_encode)
 * and derives the codes from its output.  Payloads are 16-byte aligned; strided payload rows
 * (d_payloads + i * ld_bytes, ld_bytes >= flc_payload_bytes, a multiple of 16) or a device
 * array of payload pointers.
 * -------------------------------------------------------------------------------------- */
int64_t flc_payload_bytes(const flc_codec_params* prm, int64_t d);
int flc_payload_format(const flc_codec_params* prm);
size_t flc_pack_workspace_size(const flc_codec_params* prm, int64_t d);
int flc_pack(const flc_codec_params* prm, const flc_pattern* pat, const float* d_x, int64_t d,
             void* d_payload, void* d_ws, size_t ws_bytes, void* stream);
int flc_unpack(const flc_codec_params* prm, const void* d_payload, int64_t d, float* d_out,
               void* stream);
/* Host-side check of a message received from a peer, before it goes to the device: nbytes >=
 * flc_payload_bytes, header format = the codec's, bad = 0, count = d (dense formats) / <= K with
 * strictly ascending indices < d (SPARSE) / the codec's rank (RANKK), level codes <= s (Q8 / Q16).
 * FLC_OK or FLC_ERR_ARG with the reason in flc_last_error_string.  Host memory only; no device work.
 * (The decode kernels also never index outside the row or the level table, whatever the bytes.)
 * Replaces the trust the reference's transport places in pickle.loads of the peer's reply
 * (model_funcs.py:445-452, comm_socket.py:59-82). */
int flc_payload_validate(const flc_codec_params* prm, const void* h_payload, int64_t nbytes, int64_t d);
size_t flc_unpack_reduce_workspace_size(const flc_codec_params* prm, int64_t n, int64_t d);
int flc_unpack_reduce(const flc_codec_params* prm, const void* d_payloads, int64_t ld_bytes,
                      const void* const* d_payload_ptrs, int64_t n, int64_t d, const float* d_w,
                      float w_total, float* d_out, void* d_ws, size_t ws_bytes, void* stream);

/* ----------------------------------------------------------------------------------------
 * Multi-GPU combine on a caller-owned RCCL communicator (rccl_comm: an ncclComm_t, passed as
 * void* so no RCCL type crosses the boundary).  Each rank's d_partial holds the client-order
 * partial sum of its client block (flc_encode_reduce / flc_unpack_reduce with w_total = 1.0);
 * on return every rank holds the global result:
 *   FLC_COMBINE_ALLREDUCE  in-place all-reduce(sum), then / w_total (RCCL's summation order)
 *   FLC_COMBINE_ORDERED    all-gather into d_ws, fixed rank-order fold, / w_total
 *                          (bit-reproducible; d_ws of flc_combine_workspace_size bytes)
 * Replaces the reference's per-client .to(device) gathering into one master thread
 * (thread_pool.py:59, algorithms.py:1756-1763).  Enqueued on stream; no host synchronisation.
 * -------------------------------------------------------------------------------------- */
enum { FLC_COMBINE_ALLREDUCE = 0, FLC_COMBINE_ORDERED = 1 };
size_t flc_combine_workspace_size(void* rccl_comm, int64_t d, int mode);
int flc_combine_partials(void* rccl_comm, float* d_partial, int64_t d, float w_total, int mode,
                         void* d_ws, size_t ws_bytes, void* stream);

/* G-invariant combine (SURVEY §8e "combine the 8 block partials in fixed order"): the round's
 * clients fall into fixed contiguous blocks (8 in flpytorch_amd.sharding), split evenly over the
 * ranks in rank order; d_blocks holds this rank's nb_local exact block partials (rows ld floats
 * apart, block order).  On return every rank's d_out = (((B_0 + B_1) + ...) + B_last) / w_total
 * over ALL blocks — the same bits for any rank count.  All-to-all of column slices (grouped
 * ncclSend/ncclRecv), a block-order fold of the rank's slice, ncclAllGather: per rank
 * ~2 (G-1)/G x 4 D bytes with one block per rank.  Every rank must pass the same nb_local and d.
 * Replaces the same reference code as flc_combine_partials. */
size_t flc_combine_blocks_workspace_size(void* rccl_comm, int64_t nb_local, int64_t d);
int flc_combine_blocks(void* rccl_comm, const float* d_blocks, int64_t ld, int64_t nb_local, int64_t d,
                       float w_total, float* d_out, void* d_ws, size_t ws_bytes, void* stream);

/* ----------------------------------------------------------------------------------------
 * Host side of compat mode: the numpy legacy MT19937 stream (what the reference's
 * rndgen.choice / rand / random / randint draw, compressors.py:204-212, algorithms.py:2055),
 * advanced in place on a caller-held state (key[624], pos — numpy's get_state() layout).
 * Each call consumes exactly the draws numpy would, so the caller can hand the state back
 * to its RandomState (set_state) and the experiment stream stays identical.
 * h_scratch for choice: n int64 (the Fisher-Yates array).
 * -------------------------------------------------------------------------------------- */
int flc_mt_choice(uint32_t* h_key, int32_t* h_pos, int64_t n, int64_t k, int64_t* h_out,
                  int64_t* h_scratch);
int flc_mt_rand(uint32_t* h_key, int32_t* h_pos, int64_t n, double* h_out);
int flc_mt_randint31(uint32_t* h_key, int32_t* h_pos, int64_t count, int64_t* h_out);

/* Device-RNG mode, host mirror: the uniform (a multiple of 2^-32) / the RandK index set the
 * kernels draw for (seed, client, element). */
double flc_device_uniform(uint64_t seed, int64_t client, int64_t j);
int flc_device_randk_indices(uint64_t seed, int64_t client, int64_t d, int64_t k, int64_t* h_out);
/* The device sampler's per-chunk member counts of clients client0 .. client0 + n - 1, computed by
 * the kernel the fused RandK path runs (k_randk_counts), into d_counts[C][n] (C = ceil(d / 4096),
 * uint32, chunk-major): the GPU-side check of the sampler against its host mirror and the numpy
 * restatement.  Workspace of flc_device_randk_counts_workspace_size bytes; enqueued on stream. */
size_t flc_device_randk_counts_workspace_size(int64_t n, int64_t d);
int flc_device_randk_counts(uint64_t seed, int64_t client0, int64_t n, int64_t d, int64_t k, uint32_t* d_counts,
                            void* d_ws, size_t ws_bytes, void* stream);

/* The fp32 2-norm of each of n rows (row i at d_rows + i*ld) in torch's CPU reduction order —
 * the norm the reference computes, compressors.py:272 `torch.norm(x, p=2)` on a CPU fp32
 * tensor, bit for bit ON AN x86 HOST WITH AVX2 (torch 2.10's AVX2 Vectorized<float> of 8 lanes —
 * the norm kernel has no AVX512 registration, so AVX512 hosts run it too: 8 lane accumulators of
 * fused multiply-adds summed left to right, the D % 8 tail added in order, then the correctly
 * rounded sqrt; oracle/torch_norm.c, pinned by tests/golden/rows.json at D = 25 M and against
 * torch on an AVX512 host by tests/test_host.py).  A torch without AVX2 kernels (DEFAULT
 * capability, non-x86) sums in another lane count: parity there is unpinned.  Not exactly rounded (14 616 ulp below
 * the exact norm at D = 25 M); hand it to flc_encode's d_pnorm_in to get the reference's dithering
 * bits (standard and natural dithering, compressors.py:272 / 303).  Each row is D / 8 dependent
 * fmas per lane: latency-bound (a parity mode; bench.py --dropin --norm-mode torch_cpu prices it). */
int flc_norm2_torch_cpu(const float* d_rows, int64_t ld, int64_t n, int64_t d, float* d_out, void* stream);

/* The same norms, bit for bit, without the chain (ABI 1.03): while a lane's accumulator stays in
 * one binade its rounding grid is fixed, so each step is A -> A + D(A mod 2) on that grid (two
 * integers; the parity carries ties-to-even) and runs of steps compose associatively; the steps
 * that cross a binade are taken as real fmas (torch_norm.hip).  Three launches, a workspace of
 * flc_norm2_torch_cpu_workspace_size(n, d) bytes (per row ~24 bytes per 4096 elements); n <= 65535. */
size_t flc_norm2_torch_cpu_workspace_size(int64_t n, int64_t d);
int flc_norm2_torch_cpu_ws(const float* d_rows, int64_t ld, int64_t n, int64_t d, float* d_out, void* d_ws,
                           size_t ws_bytes, void* stream);

/* Self-test of the exact fast fp32 division the dithering kernels use: for each of the n
 * device divisors, every float numerator in [2^-80, 2^80] is divided both ways and the
 * mismatches are written to d_mismatches[n] (device).  Must be all zero. */
int flc_selftest_division(const float* d_divisors, int n, unsigned long long* d_mismatches, void* stream);

/* ----------------------------------------------------------------------------------------
 * Kernel timing (off by default).  While enabled, every launch of the named hot kernels is
 * bracketed by hipEvents recorded on the launch stream; flc_profile_collect() waits for them
 * and returns the summed duration and launch count for one kernel name, then forgets them.
 * Names: k_topk_filter, k_topk_sample, k_radix_hist, k_chunk_accum, k_ew_accum_vec,
 * k_norm_partials, k_reduce_vec, k_randk_scatter; the TopK filter's variant is recorded too
 * (k_topk_filter_g4: 4-chunk work items, the many-row path of large launches; k_topk_filter_g2:
 * 2-chunk items), so a test can assert which one ran.
 * -------------------------------------------------------------------------------------- */
int flc_profile_enable(int on);
int flc_profile_collect(const char* kernel, double* h_total_ms, int64_t* h_launches);

/* Path report of the last TopK selection (test hook, no compute): copies the per-row state
 * words the previous flc_encode_reduce / flc_encode (TopK) left in d_workspace — called with the
 * same params, n and d — into d_flags[n] (device, on `stream`).  Bits: 1 the candidate list
 * overflowed, 2 it came up short, 4 ambiguous ties at the K-th key resolved on the fast path,
 * 8 the row was selected by the exact path (the fast path failed — bits 1 / 2 then say why — or
 * K > D/16), 16 a lone compressVector row (flc_encode, n = 1) selected exactly in registers in one
 * launch (rows up to 16 float4 x 4096 x the device's CUs; 4 then marks a tie cut), 32 (with 16)
 * that launch's grid was not co-resident — a grid wait gave up, the call was aborted and its last
 * workgroup re-selected the row exactly (same result).  Rows that stayed on the fast path read 0
 * or 4.  (Replaces nothing in the reference: compressors.py:330-335 has one path.) */
int flc_select_row_flags(const flc_codec_params* prm, int64_t n, int64_t d, const void* d_workspace,
                         size_t ws_bytes, uint32_t* d_flags, void* stream);

/* Host helper (no compute; the compute entries still never allocate): storage for the resident
 * client-update matrix.  contiguous != 0: physically contiguous HBM (hipDeviceMallocContiguous) —
 * a default allocation of tens of GB is stitched from fragments and some of its rows read 6-10 %
 * slower with more address-translation misses; contiguous memory maps with the largest fragments
 * (C4's shard: plain read 8.04 vs 8.48 ms, encode+reduce step 9.09 vs 9.57 ms, one process).
 * FLC_ERR_HIP when the allocation fails (e.g. no contiguous range that large is free): the caller
 * may fall back to contiguous = 0.  Free with flc_rows_free.  (The reference keeps its N client
 * tensors wherever torch puts them, model_funcs.py:367-386.) */
int flc_rows_alloc(size_t bytes, int contiguous, void** d_ptr);
int flc_rows_free(void* d_ptr);

/* Test hook of the lone-TopK resident selection (no compute): the next resident launches of this
 * process use grid_mult x their grid (grid_mult > 1: more 1024-thread workgroups than can be
 * resident at once, so the call's grid waits give up and its abort + exact repair path runs) and
 * give up a grid wait after spin_ticks of the 100 MHz clock (0: the default, 0.1 s).
 * flc_debug_resident(1, 0) restores the defaults.  FLC_ERR_ARG outside grid_mult 1..64,
 * spin_ticks >= 0.  (Replaces nothing in the reference.) */
int flc_debug_resident(int grid_mult, int64_t spin_ticks);

#ifdef __cplusplus
}
#endif
#endif /* FLCODEC_H */
