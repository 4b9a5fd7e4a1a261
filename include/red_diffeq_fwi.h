/*
 * red_diffeq_fwi.h — C ABI of the MI355X-native FWI hot path (libred_diffeq_hip.so).
 *
 * Replaces, as a drop-in boundary, the compute behind the reference's Python plugin
 * ``FWIForward`` (SimingShan/red-diffeq red_diffeq/solvers/pde.py:6-93) and the autograd
 * adjoint PyTorch derives from it (triggered at red_diffeq/core/inversion.py:86).  The Python
 * mirror of the reference interface (red-diffeq_amd/red_diffeq/solvers/pde.py) binds these
 * symbols with ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions
 *   - Plain pointers and sizes; device pointers unless stated "host".  No torch types.
 *   - Every call is stream-ordered on the given hipStream_t (NULL = legacy default stream) and
 *     returns 0 or a negative error code (-hipError_t, or RDQ_E_* below).
 *   - One call in flight per plan, enforced by the plan: its host state (graph cache, chain streams)
 *     is mutex-guarded, so any host thread may call it, and a forward / adjoint call on a different
 *     stream than the plan's previous one first waits (an event, no host sync) for the work that
 *     stream had queued, so calls on one plan never overlap on the device.  The previous call's
 *     stream must still exist at that point.  Different plans are independent.
 *   - The caller owns every buffer; sizes come from rdq_fwi_sizes().  The plan owns only the
 *     uploaded geometry (a few KB) and its cached hipGraphs.
 *   - Results are deterministic: every reduction has a fixed order.  The one float atomic, the wide
 *     chunked adjoint's fp64 add of a workgroup's sponge partial into its gk_part slot, has exactly
 *     one writer per slot and launch and no slot shared between concurrent launch chains (checked on
 *     the host for every launch of a time loop before it is enqueued; RDQ_E_INVALID otherwise), so
 *     each slot's adds arrive one launch after another in stream order: a fixed order.
 *   - Layout: padded grid Hp = nz + 2*nbc rows, Wp = nx + 2*nbc columns, row pitch `ld`
 *     floats (Wp rounded up to 64).  fp32 throughout, as the reference.
 */
#ifndef RED_DIFFEQ_FWI_H
#define RED_DIFFEQ_FWI_H

#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RDQ_E_INVALID (-10001) /* bad argument / shape */
#define RDQ_E_NOMEM (-10002)   /* host allocation failed */
#define RDQ_E_HANDOFF (-10003) /* a persistent kernel's neighbour hand-off timed out (results invalid) */

/* Acquisition geometry, host memory.  Mirrors FWIForward's ctx after __init__ and adj_sr
 * (pde.py:16-23, 54-59): all indices already on the padded grid. */
typedef struct rdq_fwi_geom {
    int32_t nz, nx;            /* model size (rows = depth, cols = width) */
    int32_t nbc;               /* sponge width, pde.py ctx['nbc'] */
    int32_t nt;                /* time steps */
    int32_t ns, ng;            /* shots, receivers */
    int32_t sample_temporal;   /* record every k-th step (pde.py:82) */
    float dx, dt;
    int32_t isz, igz;          /* source / receiver row on the padded grid */
    const int32_t *isx;        /* host [ns] source columns (padded grid) */
    const int32_t *igx;        /* host [ng] receiver columns (padded grid) */
    const double *wavelet;     /* host [nt] Ricker wavelet (pde.py:26-36), fp64 */
} rdq_fwi_geom;

typedef struct rdq_fwi_plan rdq_fwi_plan;

/* Byte sizes of the caller-owned buffers for batch B (number of velocity models). */
typedef struct rdq_fwi_sizes_t {
    int32_t Hp, Wp, ld, nrec;  /* padded grid, row pitch (floats), recorded steps */
    size_t coeffs;             /* float [6][B][Hp][ld] alpha, temp1, temp2, kappa, beta, v; then
                                  v_model [B][nz][nx] and the sponge amplitude ks [B] */
    size_t vstat;              /* float vmin[B] then int64 argmin[B] (row-major index into nz*nx) */
    size_t seis;               /* float [B][ns][nrec][ng] */
    size_t history;            /* float [nt+2][B][ns][Hp][ld]; slot j = P_{j-1} */
    size_t ring;               /* workspace, 32 B per grid cell: the chunked kernels use it as float
                                  [4][B][ns][Hp][ld] (two in/out level pairs: no-grad forward,
                                  adjoint lambdas), the persistent kernels as u64 hand-off granules
                                  [2 parity][2 level][B][ns][Hp][ld] */
    size_t gA;                 /* float [B][ns][Hp][ld] per-shot accumulator d(loss)/d(alpha) */
    size_t gk_part;            /* double [B][ns][n_adj_blocks] sponge-coefficient partial sums */
    size_t gbeta;              /* float [B][ns] source-amplitude gradient */
    size_t colsum;             /* double [B][Hp][nx] replicate-fold workspace */
} rdq_fwi_sizes_t;

/* Create / destroy a plan (uploads geometry; replaces FWIForward.__init__, pde.py:8-24). */
int rdq_fwi_plan_create(const rdq_fwi_geom *geom, rdq_fwi_plan **plan);
int rdq_fwi_plan_destroy(rdq_fwi_plan *plan);
int rdq_fwi_sizes(const rdq_fwi_plan *plan, int32_t B, rdq_fwi_sizes_t *out);
/* 1 = capture each time loop into a cached hipGraph (default), 0 = direct launches. */
int rdq_fwi_set_graphs(rdq_fwi_plan *plan, int32_t enable);
/* Time steps advanced per launch by the forward / adjoint kernels (temporal blocking depth,
 * 1..4; the wide chunked adjoint has its own depth, rdq_fwi_set_wide_adj_steps) and the number of
 * concurrent shot-group launch chains of the chunked kernels (1..16, or 0 = auto, the default: 2 for
 * the wide kernels, 1 for the 64-column ones).  Results are identical for every setting; only speed
 * changes. */
int rdq_fwi_set_tuning(rdq_fwi_plan *plan, int32_t fwd_steps, int32_t adj_steps, int32_t chains);
/* Kernel variant flags (a new plan starts at RDQ_VARIANT_FWD_GEN):
 *   RDQ_VARIANT_FWD_GEN    the chunked forward regenerates alpha/temp1/temp2 from the model in
 *                          registers instead of loading the three K3 fields (identical results;
 *                          14% faster on the configs[4] grid);
 *   RDQ_VARIANT_ADJ_EXACT  the adjoint keeps the oracle's exact fp32 operation order (gA
 *                          bit-identical to oracle/fwi_oracle.c) instead of, in the persistent
 *                          kernels, rebuilding the gradient's stencil term from the forward's time
 *                          recurrence with FMA contraction (dL/dv within ~1e-5 rel-L2) and, in the
 *                          wide chunked kernels, contracting the stencils into FMAs (dL/dv within
 *                          ~2e-5).  Plans whose sponge is thinner than 20 cells (nbc < 20) always run
 *                          the exact order: there the recurrence's cancellation is not fp32-accurate
 *                          (5e-3 at nbc = 4) and standing modes amplify any contraction;
 *   RDQ_VARIANT_NO_XCD_LOCAL the persistent kernels publish every neighbour hand-off write-through
 *                          (sc1) instead of keeping whole slices on one XCD (read from HW_REG_XCC_ID)
 *                          with L2-resident hand-offs (identical results; slower);
 *   RDQ_VARIANT_NARROW_CHUNKED the chunked (non-resident) kernels run 64-column regions, one column
 *                          per lane, instead of 128-column regions of two columns per lane
 *                          (identical results; more halo traffic);
 *   RDQ_VARIANT_CHUNKED_ADJ_FMA the wide chunked adjoint contracts its stencils into FMAs (about 4 %
 *                          faster at configs[4]; dL/dv within ~2e-5 of the oracle, the sponge sum gk,
 *                          a difference of nearly equal adjoint levels, within ~1.3e-4).  Without it
 *                          (default) the chunked adjoint keeps the oracle's exact order: gA / gbeta
 *                          bit-identical, gk to fp64 summation order.  Ignored when
 *                          RDQ_VARIANT_ADJ_EXACT is set or nbc < 20. */
#define RDQ_VARIANT_FWD_GEN 1
#define RDQ_VARIANT_ADJ_EXACT 2
#define RDQ_VARIANT_NO_XCD_LOCAL 4
#define RDQ_VARIANT_NARROW_CHUNKED 8
#define RDQ_VARIANT_CHUNKED_ADJ_FMA 16
int rdq_fwi_set_variant(rdq_fwi_plan *plan, int32_t flags);
/* Time steps per launch of the WIDE chunked adjoint (k_adj_tw, 1..6, or 0 = the default, 5: the
 * fastest depth measured at configs[4] for both the exact-order and the contracted kernels,
 * profiles/r5/configs4_wide_adj_depth.jsonl).  rdq_fwi_set_tuning's adj_steps sets the persistent and the
 * narrow chunked adjoints' depth only.  A time loop whose nt is not a multiple of the depth ends with
 * one shorter launch of its own depth.  Results are identical for every depth. */
int rdq_fwi_set_wide_adj_steps(rdq_fwi_plan *plan, int32_t steps);
/* Shots per workgroup of the WIDE chunked adjoint (1..64, or 0 = auto, the default: the cheapest of
 * 16 / 8 / 4 / 2 / 1 under rounds of one workgroup per CU x (shots + a workgroup's fixed cost)): a workgroup runs that many
 * shots of one region in turn and generates the region's alpha / kappa once for all of them.
 * Results are identical for every setting. */
int rdq_fwi_set_wide_adj_shots(rdq_fwi_plan *plan, int32_t shots);
/* The same for the WIDE chunked forward (k_fwd_tw; 0 = auto, the default). */
int rdq_fwi_set_wide_fwd_shots(rdq_fwi_plan *plan, int32_t shots);
/* Time steps per launch of the WIDE chunked forward (k_fwd_tw, 1..6, or 0 = rdq_fwi_set_tuning's
 * fwd_steps, the default).  Results are identical for every depth. */
int rdq_fwi_set_wide_fwd_steps(rdq_fwi_plan *plan, int32_t steps);
/* Rows per wave of the 64 x 96-region persistent kernels: forward 6, 8, 12 or 24 (16, 12, 8 or 4
 * waves per workgroup), adjoint (FMA build) 6, 8 or 12.  Same region geometry and results.  The time
 * step is latency-bound, so more resident waves win (configs[1], tools/ab_rw.sh, tools/ab_adj_nb6.sh):
 * forward 6 rows 1.31 ms (barrier-free exchange), 8 rows 1.40, 12 rows 1.63, 24 rows 2.42; adjoint
 * 6 rows 1.65 ms, 8 rows 1.67, 12 rows 2.08.  Default 6 / 6. */
int rdq_fwi_set_rows_per_wave(rdq_fwi_plan *plan, int32_t fwd_rows, int32_t adj_rows);
/* Delay, in 10 ns ticks (0..100000), between a persistent launch's per-epoch publish of its border and
 * its first hand-off sweep pass, for the forward and the adjoint (defaults 15 / 0 = 0.15 / 0 us: a
 * forward pass issued at once mostly finds the neighbours' granules not there yet and queues ahead of
 * the one that would; configs[1] forward 1.210 -> 1.196 ms against 0.25 us; the barrier-free adjoint
 * is fastest without a delay).  Results are identical for every delay; only speed changes. */
int rdq_fwi_set_sweep_delay(rdq_fwi_plan *plan, int32_t fwd_ticks, int32_t adj_ticks);
/* 1 (default) = run each time loop as ONE persistent launch (regions resident in registers for
 * all nt steps, epoch-wise neighbour hand-offs) whenever the whole grid fits resident on the
 * device: small surveys (at most 200 workgroups, e.g. 3 OpenFWI shots) in 64 x 64 regions of 16
 * waves x 4 rows, otherwise 64 x 96 regions if they fit, else 64 x 64 regions of 8 waves x 8 rows;
 * 16 / 12 / 8 = only that region class; 0 = always the chunked launches.  Identical results in every mode.  -1 (fault-path tests only):
 * persistent launches oversubscribed to twice the resident capacity, so they report "not resident"
 * through the status word instead of computing. */
int rdq_fwi_set_persistent(rdq_fwi_plan *plan, int32_t mode);
/* Synchronises `stream` and reports (then clears) a persistent-kernel hand-off timeout:
 * 0, or RDQ_E_HANDOFF when some launch since the last call gave up waiting for a neighbour. */
int rdq_fwi_status(rdq_fwi_plan *plan, hipStream_t stream);
/* Diagnostics (synchronises the device): the plan's 32 status words: [0] hand-off status
 * (1 = neighbour timeout, 2 = launch not resident), [16..23] workgroups per XCD of the last
 * persistent launch. */
int rdq_fwi_debug_words(rdq_fwi_plan *plan, uint32_t out[32]);
/* Caller-owned status words (device memory, >= 64 uint32, zeroed by the caller; NULL = the plan's
 * own): word 0 is non-zero once a persistent launch gave up (1 = neighbour hand-off timeout,
 * 2 = launch not resident) and stays so until the caller clears it.  Lets the caller read it
 * stream-ordered without a host sync (e.g. as the Adam guard of rdq_adam_step, or copied
 * asynchronously to pinned host memory).  Replaces the plan's internal words for later launches. */
int rdq_fwi_set_status_buffer(rdq_fwi_plan *plan, uint32_t *words);
/* Which kernels a forward / adjoint call for batch B runs: out = {forward persistent region
 * class (16 = 64 x 64 regions of 16 waves x 4 rows, 12 = 64 x 96 regions, 8 = 64 x 64 of 8 waves x 8
 * rows; 0 = chunked), the same for the adjoint, forward steps per epoch/launch,
 * adjoint steps per epoch/launch, forward time-loop launches per call, adjoint time-loop launches
 * per call} (persistent: one per resident shot group; chunked: ceil(nt / T)). */
int rdq_fwi_launch_info(rdq_fwi_plan *plan, int32_t B, int32_t out[6]);
/* The wide chunked kernels' launch shape for batch B: out = {concurrent launch chains, shots per
 * workgroup of the forward's and of the adjoint's full-depth launches of chain 0 (the automatic choice
 * unless rdq_fwi_set_wide_*_shots fixed one), shots in chain 0}. */
int rdq_fwi_wide_info(rdq_fwi_plan *plan, int32_t B, int32_t out[4]);
/* Diagnostics: 1 = the persistent kernels accumulate per-wave phase times (s_memrealtime, 10 ns
 * ticks); read_profile synchronises the device, returns and clears them:
 * out[0..5] forward {hand-off wait, time steps, publish, waves, first sweep pass, sweep passes},
 * out[6..11] the same for the adjoint. */
int rdq_fwi_set_profile(rdq_fwi_plan *plan, int32_t enable);
int rdq_fwi_read_profile(rdq_fwi_plan *plan, uint64_t out[12]);
/* Per-wave records of the last read_profile: out[(block * 16 + wave) * 3 + {0,1,2}] = {hand-off,
 * steps, publish} ticks of the forward (adj = 0) or adjoint (adj = 1) kernel. */
int rdq_fwi_profile_waves(rdq_fwi_plan *plan, int32_t adj, uint64_t *out, size_t count);

/* Velocity input convention of rdq_fwi_coeffs / rdq_fwi_grad_finalize. */
#define RDQ_VEL_NORMALIZED 0  /* v_norm in [-1,1], denormalised in-kernel: (v+1)/2*3000+1500 */
#define RDQ_VEL_PHYSICAL 1    /* velocity in m/s (FWIForward(normalize=False) or a custom denorm) */

/* K3: coefficient fields from a velocity v[b][0][iz][ix] given by element strides (any view,
 * e.g. mu[:, :, 1:-1, 1:-1]).  Replaces v_denormalize + F.pad(replicate) + get_Abc + the
 * alpha/temp1/temp2/beta lines (data_trans.py:13-15, pde.py:91, 38-52, 63-71). */
int rdq_fwi_coeffs(const rdq_fwi_plan *plan, int32_t B, const float *v, const int64_t strides[4],
                   int32_t vel_mode, float *coeffs, void *vstat, hipStream_t stream);

/* K1: forward time loop (pde.py:74-86).  history == NULL: no-grad forward; otherwise every P_j
 * is kept in `history` for the adjoint.  `ring` is the workspace (required when the persistent
 * kernel runs; the chunked history path does not touch it). */
int rdq_fwi_forward(const rdq_fwi_plan *plan, int32_t B, const float *coeffs, float *seis,
                    float *history, float *ring, hipStream_t stream);

/* K2: discrete adjoint of the forward (the autograd backward of pde.py:74-86), given
 * dseis = d(loss)/d(seis).  Writes the accumulators gA, gk_part, gbeta (overwritten).  All buffers
 * are device memory (hipMalloc / torch CUDA tensors): the wide chunked kernels add into gk_part with
 * hardware fp64 atomics, which fine-grained host memory does not support. */
int rdq_fwi_adjoint(const rdq_fwi_plan *plan, int32_t B, const float *coeffs,
                    const float *history, const float *dseis, float *ring, float *gA,
                    double *gk_part, float *gbeta, hipStream_t stream);

/* K4: d(loss)/d(v) [B][nz][nx] (contiguous) from the accumulators: chain through
 * alpha/beta/sponge(vmin), replicate-pad fold, and (RDQ_VEL_NORMALIZED) the x1500 of the
 * denormalisation. */
int rdq_fwi_grad_finalize(const rdq_fwi_plan *plan, int32_t B, const float *coeffs,
                          const void *vstat, const float *gA, const double *gk_part,
                          const float *gbeta, int32_t vel_mode, double *colsum, float *g_v,
                          hipStream_t stream);

/* K5: L1 observation loss (red_diffeq/core/losses.py:14-41), contiguous [B][n] operands.
 * forward:  loss[b] = sum(|y - pred| * mask) / nobs[b],  nobs[b] = max(sum(mask), 1)
 * backward: dpred = sign(pred - y) * mask * (gout[b] / nobs[b])       (mask NULL = all ones)
 * `partial` is a workspace of rdq_l1_partial_bytes(B, n) bytes. */
size_t rdq_l1_partial_bytes(int32_t B, int64_t n);
int rdq_l1_forward(int32_t B, int64_t n, const float *pred, const float *y, const float *mask,
                   float *loss, float *nobs, void *partial, hipStream_t stream);
int rdq_l1_backward(int32_t B, int64_t n, const float *pred, const float *y, const float *mask,
                    const float *nobs, const float *gout, float *dpred, hipStream_t stream);

/* K6: TV / Tikhonov regulariser (red_diffeq/regularization/benchmark.py:4-37) on a contiguous
 * mu[B][1][H][W].  kind: 0 = TV (mean|dx| + mean|dy|), 1 = Tikhonov (mean dx^2 + mean dy^2).
 * backward writes grad = d(sum_b gout[b] * loss[b]) / d(mu) (overwritten). */
int rdq_smooth_reg_forward(int32_t kind, int32_t B, int32_t H, int32_t W, const float *mu,
                           float *loss, hipStream_t stream);
int rdq_smooth_reg_backward(int32_t kind, int32_t B, int32_t H, int32_t W, const float *mu,
                            const float *gout, float *grad, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* RED_DIFFEQ_FWI_H */
