/*
 * red_diffeq_loop.h — C ABI of the inversion loop's serial tail (libred_diffeq_hip.so).
 *
 * Replaces the per-iteration PyTorch work around the FWI gradient in
 * SimingShan/red-diffeq red_diffeq/core/inversion.py:86-111:
 *   K11 rdq_adam_step   torch.optim.Adam.step (foreach path, amsgrad=False, weight_decay=0)
 *                       + mu.data.clamp_(-1, 1) in ONE elementwise pass (inversion.py:87-90)
 *   K12 rdq_metrics     MetricsCalculator.calculate (red_diffeq/core/metrics.py:13-46): MAE, RMSE and
 *                       SSIM (red_diffeq/utils/ssim.py:19-65, 11x11 Gaussian, sigma 1.5, zero pad)
 *                       of every model, written to a device array (no host sync per iteration)
 * fp32, caller-owned buffers, stream-ordered, deterministic (fixed-order reductions), 0 / negative
 * error codes (RDQ_E_INVALID = -10001).
 */
#ifndef RED_DIFFEQ_LOOP_H
#define RED_DIFFEQ_LOOP_H

#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One Adam step on n contiguous parameters, then clamp to [lo, hi] when clamp != 0:
 *   m = lerp(m, g, 1 - beta1);  v = v * beta2 + (1 - beta2) g g
 *   p = p + step_size * m / (sqrt(v) / bc2_sqrt + eps)
 * step_size = -lr / (1 - beta1^t) and bc2_sqrt = sqrt(1 - beta2^t) are computed by the caller in
 * double precision exactly as torch.optim.Adam does (torch/optim/adam.py, _multi_tensor_adam).
 * guard (nullable, device): when *guard != 0 the step leaves param / exp_avg / exp_avg_sq untouched
 * (the FWI status word: a gradient from a failed persistent launch is never applied). */
int rdq_adam_step(int64_t n, float *param, const float *grad, float *exp_avg, float *exp_avg_sq, float beta1,
                  float beta2, float eps, float step_size, float bc2_sqrt, int32_t clamp, float lo, float hi,
                  const uint32_t *guard, hipStream_t stream);

/* MAE, RMSE, SSIM of pred (B,1,H,W) given by element strides (any view, e.g. mu[:, :, 1:-1, 1:-1])
 * against true_norm (contiguous B,1,H,W, already v_normalize'd), SSIM on (x + 1) / 2.
 * out: float[3][B] = {mae[B], rmse[B], ssim[B]}.  ws: rdq_metrics_ws_bytes(B, H, W) bytes. */
size_t rdq_metrics_ws_bytes(int32_t B, int32_t H, int32_t W);
int rdq_metrics(int32_t B, int32_t H, int32_t W, const float *pred, const int64_t strides[4], const float *true_norm,
                float *out, void *ws, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* RED_DIFFEQ_LOOP_H */
