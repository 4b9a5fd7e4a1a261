// unet.hip — MI355X (gfx950) kernels of the RED-DiffEq U-Net epsilon-predictor.
//
// Reference: SimingShan/red-diffeq red_diffeq/models/diffusion.py (Unet 220-301 and its blocks
// 78-218, q/p math 393-429, q_sample 516-519); red_diffeq/regularization/diffusion.py:63-81.
// fp32 throughout (the reference runs the U-Net in fp32 inside the inversion).
//
//   conv2d        implicit GEMM on the fp32 matrix cores (v_mfma_f32_16x16x4_f32: exact f32 FMA
//                 chain, the same rate as the f32 VALU but one VGPR per operand per lane), with the
//                 U-Net's data movement folded into the operand gather: channel concat of skips,
//                 nearest x2 upsample, 2x2 pixel-unshuffle; bias and residual add in the epilogue.
//   group_norm    fp64 per-(sample, group) statistics from per-chunk partials, then normalise +
//                 time-conditioned scale/shift + SiLU in one pass.
//   rmsnorm / linear / sinusoidal embedding / linear & full attention / RED prologue-epilogue.
#include <hip/hip_runtime.h>
#include <atomic>

#include <cmath>
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "red_diffeq_unet.h"

namespace {

#define RDQ_CHECK(x)                                   \
    do {                                               \
        hipError_t e_ = (x);                           \
        if (e_ != hipSuccess) return -(int)e_;         \
    } while (0)
#define RDQ_E_INVALID (-10001)

using f32x4 = __attribute__((ext_vector_type(4))) float;
using f32x16 = __attribute__((ext_vector_type(16))) float;
using bf16x8 = __attribute__((ext_vector_type(8))) __bf16;

// ------------------------------------------------------------------------------------ conv2d
// Implicit GEMM on the fp32 matrix cores: D[cout][pixel] = W[cout][k] x A[k][pixel], k = (ci, ky, kx).
// A workgroup (4 waves) owns a 64 (cout) x 32 (pixel) output tile; wave w the couts 16w..16w+15 as
// two 16x16 MFMA tiles (v_mfma_f32_16x16x4_f32: exact f32 products, one VGPR per operand per lane;
// lane l supplies A[m = l&15][k = l>>4] and B[k = l>>4][n = l&15], D[m = (l>>4)*4 + r][n = l&15]).
// K is staged 32 deep through double-buffered LDS (one barrier per stage; the next stage's
// global loads are in flight during the current stage's MFMAs).  Row pitches make every operand
// read conflict-free: Ws[n][k] pitch 36 (16 n x 4 k -> 64 distinct banks), As[k][p] pitch 48.
// The U-Net's data movement is folded into the A gather (channel concat of skips, nearest x2
// upsample, 2x2 pixel-unshuffle).  Small-M layers (B = 1 at 18x18 / 9x9: K up to 6912) split K over
// blockIdx.z into fp32 partial slabs summed in a fixed order by k_conv_reduce (deterministic).
constexpr int IG_BN = 64, IG_BM = 32, IG_BK = 32;
constexpr int IG_LDW = IG_BK + 4, IG_LDA = IG_BM + 16;

struct IgArgs {
    rdq_conv_desc d;
    const float *x, *x2, *w, *bias, *res;
    float *y;                 // S == 1: output (+ bias + residual)
    float *part;              // S > 1: partial slabs [S][B][cout][HW]
    int K, M, HW, nsteps, per_split, S;
};

// A[k][pixel] of the logical input (zero padding outside the image)
template <int KH, int MODE>
__device__ __forceinline__ float ig_gather(const IgArgs &a, bool pv, int b, int oh, int ow, int k)
{
    if (!pv || k >= a.K) return 0.0f;
    const rdq_conv_desc &d = a.d;
    const int kh = KH ? KH : d.kh, kw = KH ? KH : d.kw;
    const int kk = kh * kw;
    const int ci = k / kk, r = k - ci * kk;
    const int ky = r / kw, kx = r - ky * kw;
    const int ih = oh + ky - d.pad, iw = ow + kx - d.pad;
    if ((unsigned)ih >= (unsigned)d.H || (unsigned)iw >= (unsigned)d.W) return 0.0f;
    if (MODE == RDQ_IN_UPSAMPLE2) {
        const int h2 = d.H >> 1, w2 = d.W >> 1;
        return a.x[(((size_t)b * d.cin1 + ci) * h2 + (ih >> 1)) * w2 + (iw >> 1)];
    } else if (MODE == RDQ_IN_UNSHUFFLE2) {
        const int c = ci >> 2, p1 = (ci >> 1) & 1, p2 = ci & 1;
        return a.x[(((size_t)b * (d.cin1 >> 2) + c) * (2 * d.H) + 2 * ih + p1) * (2 * d.W) + 2 * iw + p2];
    } else {
        if (ci < d.cin1) return a.x[(((size_t)b * d.cin1 + ci) * d.H + ih) * d.W + iw];
        return a.x2[(((size_t)b * d.cin2 + (ci - d.cin1)) * d.H + ih) * d.W + iw];
    }
}

// staging image of one k_conv_ig workgroup: Ws[2][IG_BN][IG_LDW], then As[2][IG_BK][IG_LDA]
constexpr int IG_SMEM = 2 * IG_BN * IG_LDW + 2 * IG_BK * IG_LDA;

// one (m tile bx, n tile by, K split) of the conv; smem = the IG_SMEM staging image
template <int KH, int MODE>
__device__ __forceinline__ void conv_ig_tile(const IgArgs &a, int bx, int by, int split, float *smem)
{
    auto &Ws = *reinterpret_cast<float (*)[2][IG_BN][IG_LDW]>(smem);
    auto &As = *reinterpret_cast<float (*)[2][IG_BK][IG_LDA]>(smem + 2 * IG_BN * IG_LDW);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int m0 = bx * IG_BM, n0 = by * IG_BN;
    const int N = a.d.cout, K = a.K;
    const int s_begin = split * a.per_split, s_end = min(a.nsteps, s_begin + a.per_split);
    // gather role: pixel gp, k rows gk + 8j
    const int gp = tid & (IG_BM - 1), gk = tid >> 5;
    const int gm = m0 + gp;
    const bool pv = gm < a.M;
    const int gb = pv ? gm / a.HW : 0, gpix = pv ? gm - gb * a.HW : 0;
    const int oh = gpix / a.d.W, ow = gpix - oh * a.d.W;
    // weight role: rows wn + 32j, k quad wk
    const int wn = tid >> 3, wk = (tid & 7) * 4;
    const bool wvec = (K & 3) == 0;
    float ra[4];
    f32x4 rw[2];
    auto load = [&](int s) {
        const int k0 = s * IG_BK;
#pragma unroll
        for (int j = 0; j < 4; ++j) ra[j] = ig_gather<KH, MODE>(a, pv, gb, oh, ow, k0 + gk + 8 * j);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int n = n0 + wn + 32 * j, k = k0 + wk;
            const float *wr = a.w + (size_t)n * K + k;
            if (n < N && wvec && k + 3 < K) {
                rw[j] = *reinterpret_cast<const f32x4 *>(wr);
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) rw[j][q] = (n < N && k + q < K) ? wr[q] : 0.0f;
            }
        }
    };
    auto stash = [&](int buf) {
#pragma unroll
        for (int j = 0; j < 4; ++j) As[buf][gk + 8 * j][gp] = ra[j];
#pragma unroll
        for (int j = 0; j < 2; ++j) *reinterpret_cast<f32x4 *>(&Ws[buf][wn + 32 * j][wk]) = rw[j];
    };
    f32x4 acc[2] = {f32x4{0.0f, 0.0f, 0.0f, 0.0f}, f32x4{0.0f, 0.0f, 0.0f, 0.0f}};
    if (s_begin < s_end) {
        load(s_begin);
        stash(0);
    }
    __syncthreads();
    for (int s = s_begin; s < s_end; ++s) {
        const int buf = (s - s_begin) & 1;
        if (s + 1 < s_end) load(s + 1);
#pragma unroll
        for (int ks = 0; ks < IG_BK / 4; ++ks) {
            const int kk = ks * 4 + (lane >> 4);
            const float av = Ws[buf][wv * 16 + (lane & 15)][kk];
            const float b0 = As[buf][kk][lane & 15], b1 = As[buf][kk][16 + (lane & 15)];
            acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b0, acc[0], 0, 0, 0);
            acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b1, acc[1], 0, 0, 0);
        }
        if (s + 1 < s_end) stash(buf ^ 1);
        __syncthreads();
    }
    const size_t slab = (size_t)a.M * N;
    // residual / bias of the 8 outputs loaded together first (clamped addresses: no per-element
    // branch), then stored: loads behind stores would be waited for one store at a time
    float rv[2][4], bv[2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int m = min(m0 + j * 16 + (lane & 15), a.M - 1);
        const int b = m / a.HW, pix = m - b * a.HW;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int n = min(n0 + wv * 16 + (lane >> 4) * 4 + r, N - 1);
            rv[j][r] = (a.S == 1 && a.res) ? a.res[((size_t)b * N + n) * a.HW + pix] : 0.0f;
            bv[j][r] = (a.S == 1 && a.bias) ? a.bias[n] : 0.0f;
        }
    }
    float ov[2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            ov[j][r] = a.S == 1 ? (acc[j][r] + bv[j][r]) + rv[j][r] : acc[j][r];
            asm volatile("" : "+v"(ov[j][r]));        // formed before any conditional store
        }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int m = m0 + j * 16 + (lane & 15);
        if (m >= a.M) continue;
        const int b = m / a.HW, pix = m - b * a.HW;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int n = n0 + wv * 16 + (lane >> 4) * 4 + r;
            if (n >= N) continue;
            const size_t o = ((size_t)b * N + n) * a.HW + pix;
            if (a.S == 1) a.y[o] = ov[j][r];
            else a.part[split * slab + o] = ov[j][r];
        }
    }
}

template <int KH, int MODE>
__global__ __launch_bounds__(256, 2) void k_conv_ig(IgArgs a)
{
    __shared__ __attribute__((aligned(16))) float sm[IG_SMEM];
    conv_ig_tile<KH, MODE>(a, blockIdx.x, blockIdx.y, blockIdx.z, sm);
}

// split-K combine: fixed slab order, then bias and residual
__global__ __launch_bounds__(256) void k_conv_reduce(int S, int64_t total, int N, int HW, const float *__restrict__ part,
                                                     const float *__restrict__ bias, const float *__restrict__ res,
                                                     float *__restrict__ y)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    float v = part[i];
    for (int s = 1; s < S; ++s) v += part[(size_t)s * total + i];
    if (bias) v = v + bias[(i / HW) % N];
    if (res) v = v + res[i];
    y[i] = v;
}

// ------------------------------------------------------------------ conv2d, channel-chunk form
// The same implicit GEMM for the U-Net's own shapes (3x3 or 1x1 filters, channel counts multiples
// of the chunk): one K stage = CPS whole input channels x every filter tap (k = ci*TAPS + tap, the
// weights' own order, so the MFMA chain visits k in the same ascending groups of 4 as k_conv_ig).
// A thread gathers the taps of ONE (pixel, channel) per stage from tap offsets and a padding mask
// computed once per launch: the per-element index arithmetic of k_conv_ig's gather is gone.  Loads
// run two stages ahead (two register sets, straight-line code so the waitcnt before a stash leaves
// the younger stage in flight) into double-buffered LDS: at B = 1 a workgroup is alone on its CU,
// so the K loop is latency-bound unless more than one stage is in flight.
// Split-K partial slabs are combined by the LAST-arriving workgroup of each tile (an arrival ticket
// per tile, then the slabs summed in slab order, then bias and residual: the arithmetic of
// k_conv_reduce, bit for bit) instead of a separate launch.  Tickets are zero before the launch and
// returned to zero by the combining workgroup.
// GroupNorm-normalised value -> affine -> time scale/shift -> SiLU (Block.forward, diffusion.py:142-149)
__device__ __forceinline__ float gn_silu1(float x, float mean, float rstd, float ga, float be, bool sso, float sc1,
                                          float sh)
{
    float v = (x - mean) * rstd;
    v = v * ga + be;
    if (sso) v = v * sc1 + sh;
    return v / (1.0f + expf(-v));
}

// element loads of a normalise pass's input: fp32, or the bf16 halo-staged conv's raw output
__device__ __forceinline__ float ldx(const float *p) { return *p; }
__device__ __forceinline__ float ldx(const __bf16 *p) { return (float)*p; }
__device__ __forceinline__ float4 ldx4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ __forceinline__ float4 ldx4(const __bf16 *p)
{
    const uint2 u = *reinterpret_cast<const uint2 *>(p);
    return float4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                  __uint_as_float(u.y & 0xffff0000u)};
}

template <int TAPS> struct CcCfg;
template <> struct CcCfg<9> { static constexpr int CPS = 8, BK = 72, NA = 9, QPR = 18, NWQ = 5; };
template <> struct CcCfg<1> { static constexpr int CPS = 64, BK = 64, NA = 8, QPR = 16, NWQ = 4; };
constexpr int CC_BN = 64, CC_BM = 32, CC_LDA = CC_BM + 16;
#ifndef RDQ_CC_WPOL
#define RDQ_CC_WPOL 0          // cache policy of the implicit-GEMM conv's weight loads
#endif
#ifndef RDQ_CC_APOL
#define RDQ_CC_APOL 0          // ... and of its activation loads
#endif
constexpr int CC_SC1 = 16;             // buffer cache policy sc1: write-through stores, L1-bypassing loads
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));

struct CcArgs {
    rdq_conv_desc d;
    const float *x, *x2, *w, *bias, *res;
    float *y, *part;
    unsigned *tickets;        // S > 1: one per (m tile, n tile)
    double *gnp;              // non-null: GroupNorm(G) partial statistics per (m tile, group, slot)
    const float *rms_g;       // RMS: the input is RMSNorm'd per pixel as it is gathered (1x1, no concat)
    int K, M, HW, nstages, per_split, S, G;
    int xbytes, x2bytes, wbytes;   // buffer extents (< 2^31: cc_ok)
};

// operand staging image of one workgroup (the 3x3 layout, the larger of the two)
constexpr int CC_SMEM = 2 * CC_BN * (CcCfg<9>::BK + 4) + 2 * CcCfg<9>::BK * CC_LDA;

// one (m tile bx, n tile by, K split) of the conv on a gx x gy tile grid; smem = the CC_SMEM staging image
// stages [s_begin, s_end) of tile (bx, by) on a gx x gy tile grid, as piece `split` of S pieces whose
// slabs the last-arriving piece sums in piece order (S == 1: the whole K range, direct epilogue;
// S < 0: slabs only, for k_conv_reduce); smem = the CC_SMEM staging image
template <int TAPS, int MODE, bool RMS>
__device__ __forceinline__ void conv_cc_seg(const CcArgs &a, int bx, int by, int s_begin, int s_end, int S, int split,
                                            int gx, int gy, float *smem)
{
    using C = CcCfg<TAPS>;
    constexpr int BK = C::BK, NA = C::NA, NWQ = C::NWQ, QPR = C::QPR, LDW = BK + 4;
    static_assert(2 * CC_BN * LDW + 2 * BK * CC_LDA <= CC_SMEM, "staging image");
    auto &Ws = *reinterpret_cast<float (*)[2][CC_BN][LDW]>(smem);
    auto &As = *reinterpret_cast<float (*)[2][BK][CC_LDA]>(smem + 2 * CC_BN * LDW);
    __shared__ unsigned last_s;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int m0 = bx * CC_BM, n0 = by * CC_BN;
    const rdq_conv_desc &d = a.d;
    const int N = d.cout, K = a.K;
    // gather role: pixel gp, channel lane cl of the stage's chunk
    const int gp = tid & (CC_BM - 1), cl = tid >> 5;
    const int gm = m0 + gp;
    const bool pv = gm < a.M;
    const int gb = pv ? gm / a.HW : 0, gpix = pv ? gm - gb * a.HW : 0;
    const int oh = gpix / d.W, ow = gpix - oh * d.W;
    // every load is a buffer load: a per-lane byte offset fixed for the launch (sample, channel
    // lane, tap; padding taps get an offset past the buffer, which loads 0) plus a wave-uniform
    // per-stage channel offset, so a stage issues its loads with no address arithmetic
    constexpr int OOB_OFF = (int)0x80000000u;
    const int plane = MODE == RDQ_IN_UPSAMPLE2 ? (d.H >> 1) * (d.W >> 1)
                    : MODE == RDQ_IN_UNSHUFFLE2 ? 4 * a.HW : a.HW;
    const int cin1 = MODE == RDQ_IN_UNSHUFFLE2 ? d.cin1 >> 2 : d.cin1;
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(a.x), (short)0,
                                                                        a.xbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rx2 = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(a.x2 ? a.x2 : a.x),
                                                                         (short)0, a.x2bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rwt = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(a.w), (short)0,
                                                                         a.wbytes, 0x00020000);
    int vo1[NA], vo2[NA];
    if constexpr (TAPS == 9) {
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const int ih = oh + t / 3 - d.pad, iw = ow + t % 3 - d.pad;
            const bool ok = pv && (unsigned)ih < (unsigned)d.H && (unsigned)iw < (unsigned)d.W;
            const int o = MODE == RDQ_IN_UPSAMPLE2 ? (ih >> 1) * (d.W >> 1) + (iw >> 1) : ih * d.W + iw;
            vo1[t] = ok ? ((gb * cin1 + cl) * plane + o) * 4 : OOB_OFF;
            vo2[t] = ok ? ((gb * d.cin2 + cl) * a.HW + o) * 4 : OOB_OFF;
        }
    } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int c = cl + 8 * j;                 // channel within the 64-channel stage
            if constexpr (MODE == RDQ_IN_UNSHUFFLE2) {
                const int o = (2 * oh + ((c >> 1) & 1)) * (2 * d.W) + 2 * ow + (c & 1);
                vo1[j] = pv ? ((gb * cin1 + (c >> 2)) * plane + o) * 4 : OOB_OFF;
            } else {
                vo1[j] = pv ? ((gb * cin1 + c) * plane + gpix) * 4 : OOB_OFF;
            }
            vo2[j] = pv ? ((gb * d.cin2 + c) * a.HW + gpix) * 4 : OOB_OFF;
        }
    }
    // weight role: quad q of row n for idx = tid + 256 r (rows past cout clamped: their outputs are
    // never stored; idx past the tile only loads, never stashes)
    int vw[NWQ];
#pragma unroll
    for (int r = 0; r < NWQ; ++r) {
        const int idx = min(tid + 256 * r, CC_BN * QPR - 1);
        const int n = idx / QPR, q = idx - n * QPR;
        vw[r] = (min(n0 + n, N - 1) * K + q * 4) * 4;
    }
    auto load = [&](int s, float (&ra)[NA], f32x4 (&rw)[NWQ]) {
        // stage s = channels [s*CPS, (s+1)*CPS): all in x or all in x2 (cin1 % CPS == 0)
        const int c0 = s * C::CPS;
        const bool first = c0 < d.cin1;
        const int soff = first ? (MODE == RDQ_IN_UNSHUFFLE2 ? (c0 >> 2) : c0) * plane * 4 : (c0 - d.cin1) * a.HW * 4;
        const __amdgpu_buffer_rsrc_t rs = first ? rx : rx2;
#pragma unroll
        for (int t = 0; t < NA; ++t)
            ra[t] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, first ? vo1[t] : vo2[t], soff, RDQ_CC_APOL));
#pragma unroll
        for (int r = 0; r < NWQ; ++r)
            rw[r] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rwt, vw[r], s * BK * 4, RDQ_CC_WPOL));
    };
    // RMS: per-pixel 1 / max(||x||, eps) from a pass over all input channels (sums of squares per
    // channel lane in channel order, combined over the 8 lanes in order), g staged in LDS
    __shared__ float rms_part[RMS ? 8 : 1][CC_BM];
    __shared__ float rms_gs[RMS ? 2048 : 1];
    float rms_den = 1.0f;
    const float rms_sc = RMS ? sqrtf((float)d.cin1) : 1.0f;
    if constexpr (RMS)
        for (int c = tid; c < d.cin1; c += 256) rms_gs[c] = a.rms_g[c];
    // (run after the pipeline's first stage loads are issued: one memory round trip for both)
    auto rms_pass = [&]() {
    if constexpr (RMS) {
        // all of the thread's channels (cl + 8j + 64i, up to 512 input channels) in flight at once;
        // channels past cin1 read 0 (offset past the buffer)
        float ssum = 0.0f;
        for (int c00 = 0; c00 < d.cin1; c00 += 512) {
            float v[64];
#pragma unroll
            for (int k = 0; k < 64; ++k) {
                const int c0 = c00 + (k >> 3) * 64;
                v[k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                    rx, vo1[k & 7], c0 < d.cin1 ? c0 * plane * 4 : a.xbytes, 0));
            }
#pragma unroll
            for (int k = 0; k < 64; ++k) ssum += v[k] * v[k];
        }
        rms_part[cl][gp] = ssum;
        __syncthreads();
        float tot = 0.0f;
#pragma unroll
        for (int k = 0; k < 8; ++k) tot += rms_part[k][gp];
        rms_den = fmaxf(sqrtf(tot), 1e-12f);
    }
    };
    auto stash = [&](int buf, int s, const float (&ra)[NA], const f32x4 (&rw)[NWQ]) {
        if constexpr (TAPS == 9) {
#pragma unroll
            for (int t = 0; t < 9; ++t) As[buf][cl * 9 + t][gp] = ra[t];
        } else if constexpr (RMS) {
            // F.normalize(x, dim=1) * g * sqrt(C), the operation order of k_rmsnorm
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float v = ra[j] / rms_den;
                v = v * rms_gs[s * C::CPS + cl + 8 * j];
                As[buf][cl + 8 * j][gp] = v * rms_sc;
            }
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) As[buf][cl + 8 * j][gp] = ra[j];
        }
#pragma unroll
        for (int r = 0; r < NWQ; ++r) {
            const int idx = tid + 256 * r;
            if (idx < CC_BN * QPR) {
                const int n = idx / QPR, q = idx - n * QPR;
                *reinterpret_cast<f32x4 *>(&Ws[buf][n][q * 4]) = rw[r];
            }
        }
    };
    f32x4 acc[2] = {f32x4{0.0f, 0.0f, 0.0f, 0.0f}, f32x4{0.0f, 0.0f, 0.0f, 0.0f}};
    // operands of a stage read from LDS in batches of BT k-groups, the next batch's reads issued
    // before the current batch's MFMAs (one wave per SIMD at B = 1: nothing else hides LDS latency)
    auto mma = [&](int buf) {
        constexpr int KS = BK / 4, BT = KS % 3 == 0 ? 3 : 4, NB = KS / BT;
        float av[2][BT], b0[2][BT], b1[2][BT];
        auto rd = [&](int bt, float (&a_)[BT], float (&x_)[BT], float (&y_)[BT]) {
#pragma unroll
            for (int u = 0; u < BT; ++u) {
                const int kk = (bt * BT + u) * 4 + (lane >> 4);
                a_[u] = Ws[buf][wv * 16 + (lane & 15)][kk];
                x_[u] = As[buf][kk][lane & 15];
                y_[u] = As[buf][kk][16 + (lane & 15)];
            }
        };
        // (sched_barrier: the machine scheduler would otherwise move each read next to its MFMA
        // and wait for it there, lgkmcnt(0) per k-group)
        rd(0, av[0], b0[0], b1[0]);
#pragma unroll
        for (int bt = 0; bt < NB; ++bt) {
            if (bt + 1 < NB) rd(bt + 1, av[(bt + 1) & 1], b0[(bt + 1) & 1], b1[(bt + 1) & 1]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < BT; ++u) {
                acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[bt & 1][u], b0[bt & 1][u], acc[0], 0, 0, 0);
                acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[bt & 1][u], b1[bt & 1][u], acc[1], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    const int ns = s_end - s_begin;
    if (ns > 0) {
        // four register sets: at step i LDS buffer i&1 holds stage i, stages i+1..i+3 are in flight
        // (three steps of MFMA work cover a load's latency), stage i+1 is stashed at the step's end
        float ra0[NA], ra1[NA], ra2[NA], ra3[NA];
        f32x4 rw0[NWQ], rw1[NWQ], rw2[NWQ], rw3[NWQ];
        const int sl = s_end - 1;         // loads past the split's end re-read its last stage
        load(s_begin, ra0, rw0);
        load(min(s_begin + 1, sl), ra1, rw1);
        load(min(s_begin + 2, sl), ra2, rw2);
        rms_pass();
        stash(0, s_begin, ra0, rw0);
        __syncthreads();
        auto step = [&](int i, float (&rl)[NA], f32x4 (&wl)[NWQ], const float (&rs)[NA], const f32x4 (&wsr)[NWQ]) {
            load(min(s_begin + i + 3, sl), rl, wl);
            mma(i & 1);
            stash((i + 1) & 1, min(s_begin + i + 1, sl), rs, wsr);
            __syncthreads();
        };
        for (int i = 0;; i += 4) {
            step(i, ra3, rw3, ra1, rw1);
            if (i + 1 >= ns) break;
            step(i + 1, ra0, rw0, ra2, rw2);
            if (i + 2 >= ns) break;
            step(i + 2, ra1, rw1, ra3, rw3);
            if (i + 3 >= ns) break;
            step(i + 3, ra2, rw2, ra0, rw0);
            if (i + 4 >= ns) break;
        }
    }
    // outputs of this lane: (n = n0 + wv*16 + (lane>>4)*4 + r, m = m0 + j*16 + (lane&15))
    if (S < 0) {                         // slabs [S][B][cout][HW] for k_conv_reduce
        const size_t slab = (size_t)a.M * N;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int m = m0 + j * 16 + (lane & 15);
            const int b = m / a.HW, pix = m - b * a.HW;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int n = n0 + wv * 16 + (lane >> 4) * 4 + r;
                if (m < a.M && n < N) a.part[split * slab + ((size_t)b * N + n) * a.HW + pix] = acc[j][r];
            }
        }
        return;
    }
    if (S > 1) {
        // in-launch combine.  Slabs in the tile's own register order (lane tid's 8 accumulators as
        // two 16-B words), written and read write-through (sc1) so no L2 fence is needed:
        // every storing wave drains its stores, the workgroup barrier, one agent-scope ticket add per
        // workgroup, and the workgroup whose add returns S-1 reads all S slabs with sc1 loads
        // (MI355X_MICROARCH.md, hand-offs with sc1 loads in place of the acquire, first row).
        const int ntile = gx * gy, tile = by * gx + bx;
        const __amdgpu_buffer_rsrc_t pr = __builtin_amdgcn_make_buffer_rsrc(a.part, (short)0, 0x7fffffff, 0x00020000);
        const int voff = tid * 32;
        const int tbase = tile * (CC_BM * CC_BN * 4);
        const int sbytes = ntile * (CC_BM * CC_BN * 4);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, acc[0]), pr, voff, split * sbytes + tbase, CC_SC1);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, acc[1]), pr, voff + 16, split * sbytes + tbase, CC_SC1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        unsigned *tk = a.tickets + tile;
        if (tid == 0) last_s = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(S - 1);
        __syncthreads();
        if (!last_s) return;
        // slabs summed in slab order, four slabs' loads in flight at a time
        f32x4 v0 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(pr, voff, tbase, CC_SC1));
        f32x4 v1 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(pr, voff + 16, tbase, CC_SC1));
        int s = 1;
        for (; s + 4 <= S; s += 4) {
            f32x4 t0[4], t1[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                t0[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(pr, voff, (s + u) * sbytes + tbase, CC_SC1));
                t1[u] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(pr, voff + 16, (s + u) * sbytes + tbase, CC_SC1));
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) { v0 += t0[u]; v1 += t1[u]; }
        }
        for (; s < S; ++s) {
            v0 += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(pr, voff, s * sbytes + tbase, CC_SC1));
            v1 += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(pr, voff + 16, s * sbytes + tbase, CC_SC1));
        }
        acc[0] = v0;
        acc[1] = v1;
        if (tid == 0) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // epilogue: (sum + bias) + residual
    float rv[2][4], bv[2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int m = min(m0 + j * 16 + (lane & 15), a.M - 1);
        const int b = m / a.HW, pix = m - b * a.HW;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int n = min(n0 + wv * 16 + (lane >> 4) * 4 + r, N - 1);
            rv[j][r] = a.res ? a.res[((size_t)b * N + n) * a.HW + pix] : 0.0f;
            bv[j][r] = a.bias ? a.bias[n] : 0.0f;
        }
    }
    float ov[2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int m = m0 + j * 16 + (lane & 15);
        const int b = m / a.HW, pix = m - b * a.HW;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int n = n0 + wv * 16 + (lane >> 4) * 4 + r;
            float v = acc[j][r];
            if (a.bias) v = v + bv[j][r];
            if (a.res) v = v + rv[j][r];
            ov[j][r] = v;
            if (m < a.M && n < N) a.y[((size_t)b * N + n) * a.HW + pix] = v;
        }
    }
    if (!a.gnp) return;
    // GroupNorm statistics of the tile's outputs, fp64 sum and sum of squares per (group, sample
    // slot: 0 = the sample of the tile's first pixel, 1 = the next; HW >= 32 so at most two), by
    // fixed trees: a lane's 4 channels (one group, C/G >= 8) per pixel, xor over the 16 pixel lanes,
    // over the lanes' 4-channel blocks of the same group, then over the waves of a group in wave
    // order; written to gnp[((m tile * G + g) * 2 + slot) * 2 + {0, 1}]
    const int cpg = N / a.G, b0 = m0 / a.HW;
    double gs[2] = {0.0, 0.0}, gq[2] = {0.0, 0.0};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int m = m0 + j * 16 + (lane & 15);
        int sl = m < a.M ? m / a.HW - b0 : -1;
        double s1 = 0.0, q1 = 0.0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const double xv = ov[j][r];
            s1 += xv;
            q1 += xv * xv;
        }
        if (n0 + wv * 16 + (lane >> 4) * 4 >= N) sl = -1;
        gs[0] += sl == 0 ? s1 : 0.0;
        gq[0] += sl == 0 ? q1 : 0.0;
        gs[1] += sl == 1 ? s1 : 0.0;
        gq[1] += sl == 1 ? q1 : 0.0;
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            gs[k] += __shfl_xor(gs[k], o, 64);
            gq[k] += __shfl_xor(gq[k], o, 64);
        }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        gs[k] += __shfl_xor(gs[k], 16, 64);          // 4-channel blocks (0,1) and (2,3): 8 channels
        gq[k] += __shfl_xor(gq[k], 16, 64);
    }
    if (cpg >= 16) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            gs[k] += __shfl_xor(gs[k], 32, 64);      // the wave's 16 channels
            gq[k] += __shfl_xor(gq[k], 32, 64);
        }
    }
    __shared__ double gpart[4][2][2][2];              // [wave][8-channel half][slot][s, q]
    if ((lane & 31) == 0) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            gpart[wv][lane >> 5][k][0] = gs[k];
            gpart[wv][lane >> 5][k][1] = gq[k];
        }
    }
    __syncthreads();
    const int gt = CC_BN / cpg;
    if (tid < 2 * gt) {
        const int g = tid >> 1, k = tid & 1;
        double s = 0.0, q = 0.0;
        if (cpg == 8) {
            s = gpart[g >> 1][g & 1][k][0];
            q = gpart[g >> 1][g & 1][k][1];
        } else {
            const int wpg = cpg / 16;
            for (int w = g * wpg; w < (g + 1) * wpg; ++w) {
                s += gpart[w][0][k][0];
                q += gpart[w][0][k][1];
            }
        }
        if (n0 + g * cpg < N) {
            double *o = a.gnp + (((size_t)bx * a.G + n0 / cpg + g) * 2 + k) * 2;
            o[0] = s;
            o[1] = q;
        }
    }
}

template <int TAPS, int MODE, bool RMS>
__device__ __forceinline__ void conv_cc_tile(const CcArgs &a, int bx, int by, int split, int gx, int gy, float *smem)
{
    const int s_begin = split * a.per_split, s_end = min(a.nstages, s_begin + a.per_split);
    conv_cc_seg<TAPS, MODE, RMS>(a, bx, by, s_begin, s_end, a.S, split, gx, gy, smem);
}

template <int TAPS, int MODE, bool RMS = false>
__global__ __launch_bounds__(256, 2) void k_conv_cc(CcArgs a)
{
    __shared__ __attribute__((aligned(16))) float sm[CC_SMEM];
    conv_cc_tile<TAPS, MODE, RMS>(a, blockIdx.x, blockIdx.y, blockIdx.z, gridDim.x, gridDim.y, sm);
}

// A ResnetBlock with a 1x1 shortcut (the U-Net's up path and final block, diffusion.py:160-168):
// block1's 3x3 conv (GroupNorm statistics in its epilogue) and res_conv of the same concatenated
// input in ONE launch: n tiles [0, gy_a) run the 3x3 tile, the rest the 1x1 tile (each with its own
// arguments, split count and tickets; the split slices past a conv's own count return at once).
// Both tiles are those of the separate launches, so the outputs are bit for bit theirs.
__global__ __launch_bounds__(256, 2) void k_conv_cc_pair(CcArgs a, CcArgs b, int gy_a)
{
    __shared__ __attribute__((aligned(16))) float sm[CC_SMEM];
    const int by = blockIdx.y, bz = blockIdx.z;
    if (by < gy_a) {
        if (bz < a.S) conv_cc_tile<9, RDQ_IN_PLAIN, false>(a, blockIdx.x, by, bz, gridDim.x, gy_a, sm);
    } else if (bz < b.S) {
        conv_cc_tile<1, RDQ_IN_PLAIN, false>(b, blockIdx.x, by - gy_a, bz, gridDim.x, gridDim.y - gy_a, sm);
    }
}

// channel-chunk form applies: 3x3 (any pad) or 1x1 (pad 0) filters, every channel count a multiple
// of the chunk (so a stage never straddles the concat seam), 16-B aligned weight rows
bool cc_ok(const rdq_conv_desc *d)
{
    const int cin = d->cin1 + d->cin2;
    if (d->kh != d->kw || (d->kh != 3 && d->kh != 1)) return false;
    const int cps = d->kh == 3 ? CcCfg<9>::CPS : CcCfg<1>::CPS;
    if (d->kh == 1 && d->pad != 0) return false;
    if (d->in_mode == RDQ_IN_UNSHUFFLE2 && d->kh != 1) return false;
    if (d->cin1 % cps || d->cin2 % cps || cin % 4) return false;
    const int64_t lim = INT32_MAX;                 // buffer-load extents and offsets are 32-bit
    const int64_t xy = (int64_t)d->B * d->H * d->W * 4;
    return xy * d->cin1 < lim && xy * d->cin2 < lim && (int64_t)d->cout * cin * d->kh * d->kw * 4 < lim &&
           xy * d->cout < lim;
}

void cc_extents(CcArgs &c, const rdq_conv_desc *d)
{
    const int64_t xy = (int64_t)d->B * d->H * d->W * 4;
    c.xbytes = (int)(d->in_mode == RDQ_IN_UPSAMPLE2 ? xy / 4 * d->cin1 : xy * d->cin1);
    c.x2bytes = (int)(xy * d->cin2);
    c.wbytes = (int)((int64_t)d->cout * c.K * 4);
}

// splits: fill the chip with about one workgroup per CU, >= 3 stages per split (the pipeline's fill),
// at most 16 slabs to combine; a grid of 128..255 tiles (half the CUs idle, or one workgroup
// per CU with nothing to hide its waits) is split in two when each half keeps >= 6 stages (a
// second workgroup on a CU shares the matrix unit but hides the first one's load / LDS latency:
// level-9 512-channel convs at B = 8 measured 73 -> see DESIGN.md)
static std::atomic<int> CC_MIN_STAGES{3};     // least K stages per split (RDQ_UNET_OPT_CC_MIN_STAGES)
static std::atomic<int> CC_SPLIT2_STAGES{12}; // 128..255 tiles split in two from this many stages (RDQ_UNET_OPT_CC_SPLIT2_STAGES)
int cc_splits(const rdq_conv_desc *d, size_t ws_bytes, int *per_split)
{
    const int M = d->B * d->H * d->W;
    const int tiles = ((M + CC_BM - 1) / CC_BM) * ((d->cout + CC_BN - 1) / CC_BN);
    const int nstages = (d->cin1 + d->cin2) / (d->kh == 3 ? CcCfg<9>::CPS : CcCfg<1>::CPS);
    int S = std::max(1, std::min(std::min(256 / tiles, nstages / std::max(1, CC_MIN_STAGES.load())), 16));
    if (tiles >= 128 && tiles < 256 && nstages >= CC_SPLIT2_STAGES.load()) S = 2;
    const size_t slab = (size_t)tiles * CC_BM * CC_BN * sizeof(float);      // >= M * cout floats
    if (S > 1) S = (int)std::min<size_t>((size_t)S, ws_bytes / slab);
    S = std::max(S, 1);
    const int per = (nstages + S - 1) / S;
    *per_split = per;
    return (nstages + per - 1) / per;
}

// split count: about one workgroup per CU over the tile grid, >= 4 K stages per split, and the
// partial slabs within the caller's workspace
int ig_splits(const rdq_conv_desc *d, size_t ws_bytes, int *per_split)
{
    const int M = d->B * d->H * d->W, K = (d->cin1 + d->cin2) * d->kh * d->kw;
    const int tiles = ((M + IG_BM - 1) / IG_BM) * ((d->cout + IG_BN - 1) / IG_BN);
    const int nsteps = (K + IG_BK - 1) / IG_BK;
    int S = std::max(1, std::min((256 + tiles - 1) / tiles, nsteps / 4));
    const size_t slab = (size_t)M * d->cout * sizeof(float);
    if (S > 1 && ws_bytes < 2 * slab) S = 1;
    if (S > 1) S = std::min<int64_t>(S, (int64_t)(ws_bytes / slab));
    const int per = (nsteps + S - 1) / S;
    *per_split = per;
    return (nsteps + per - 1) / per;
}

// -------------------------------------------------------------------------------- group norm
constexpr int GN_CHUNK = 4096;   // elements per statistics partial

__global__ __launch_bounds__(256) void k_gn_partial(const float *__restrict__ x, int64_t gsize, int nchunk,
                                                    double *__restrict__ part)
{
    const int bg = blockIdx.y, c = blockIdx.x;
    const float *p = x + (size_t)bg * gsize;
    const int64_t e0 = (int64_t)c * GN_CHUNK, e1 = min((int64_t)(c + 1) * GN_CHUNK, gsize);
    // the thread's GN_CHUNK / 256 elements are loaded together (clamped index, zero past the end),
    // then accumulated in the same order as a strided loop would
    float xv[GN_CHUNK / 256];
#pragma unroll
    for (int u = 0; u < GN_CHUNK / 256; ++u) xv[u] = p[min(e0 + threadIdx.x + 256 * u, e1 - 1)];
    double s = 0.0, q = 0.0;
#pragma unroll
    for (int u = 0; u < GN_CHUNK / 256; ++u) {
        if (e0 + threadIdx.x + 256 * u < e1) {
            const double v = xv[u];
            s += v;
            q += v * v;
        }
    }
    __shared__ double ss[256], sq[256];
    ss[threadIdx.x] = s;
    sq[threadIdx.x] = q;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) { ss[threadIdx.x] += ss[threadIdx.x + w]; sq[threadIdx.x] += sq[threadIdx.x + w]; }
        __syncthreads();
    }
    if (threadIdx.x == 0) { part[((size_t)bg * nchunk + c) * 2] = ss[0]; part[((size_t)bg * nchunk + c) * 2 + 1] = sq[0]; }
}

// mean and 1/std of (sample, group) bg from the fixed-order fp64 chunk partials
__device__ __forceinline__ void gn_stat_of(int bg, int nchunk, int64_t gsize, float eps, const double *part,
                                           float &mean_f, float &rstd_f)
{
    double s = 0.0, q = 0.0;
    for (int c = 0; c < nchunk; ++c) { s += part[((size_t)bg * nchunk + c) * 2]; q += part[((size_t)bg * nchunk + c) * 2 + 1]; }
    const double mean = s / (double)gsize;
    double var = q / (double)gsize - mean * mean;
    var = var < 0.0 ? 0.0 : var;
    mean_f = (float)mean;
    rstd_f = (float)(1.0 / sqrt(var + (double)eps));
}
// ... once per (sample, group), for large grids (the apply's workgroups then read two floats)
__global__ __launch_bounds__(256) void k_gn_stats(int BG, int nchunk, int64_t gsize, float eps,
                                                  const double *__restrict__ part, float *__restrict__ stat)
{
    const int bg = blockIdx.x * blockDim.x + threadIdx.x;
    if (bg >= BG) return;
    gn_stat_of(bg, nchunk, gsize, eps, part, stat[2 * bg], stat[2 * bg + 1]);
}

// y = SiLU(((x - mean) rstd gamma + beta) (scale + 1) + shift), one workgroup per (channel row,
// 1024-element chunk; the pass is VALU-bound on the exact expf and division of SiLU): the channel's constants are wave-uniform, four elements per lane (float4
// where the row allows it); the operation order is the per-element formula's
// stat == nullptr (small grids, where one more launch costs more than the arithmetic): every
// workgroup derives its group's statistics from the chunk partials itself
template <bool SMALL>
__global__ __launch_bounds__(256) void k_gn_apply(int C, int HW, int G, int nch, const float *__restrict__ x,
                                                  const float *__restrict__ gamma, const float *__restrict__ beta,
                                                  const float *__restrict__ ss, const float *__restrict__ stat,
                                                  const double *__restrict__ part, int nchunk, float eps,
                                                  float *__restrict__ y)
{
    const int bg = blockIdx.y, b = bg / G, g = bg - b * G, cpg = C / G;
    const int cl = SMALL ? 0 : blockIdx.x / nch, ch = SMALL ? 0 : blockIdx.x - cl * nch;
    const int c = g * cpg + cl;
    float mean, rstd;
    if (stat) {
        mean = stat[2 * bg];
        rstd = stat[2 * bg + 1];
    } else {
        __shared__ float st2[2];
        if (threadIdx.x == 0) gn_stat_of(bg, nchunk, (int64_t)cpg * HW, eps, part, st2[0], st2[1]);
        __syncthreads();
        mean = st2[0];
        rstd = st2[1];
    }
    const bool sso = ss != nullptr;
    if constexpr (SMALL) {        // small images: -nch whole channels of the group per workgroup
        const int cpb = -nch, cl0 = blockIdx.x * cpb, n = min(cpb, cpg - cl0) * HW;
        const size_t base = ((size_t)b * C + g * cpg + cl0) * HW;
        for (int e = threadIdx.x; e < n; e += 256) {
            const int cc = g * cpg + cl0 + e / HW;
            const float s1 = sso ? ss[(size_t)b * 2 * C + cc] + 1.0f : 0.0f, sh1 = sso ? ss[(size_t)b * 2 * C + C + cc] : 0.0f;
            y[base + e] = gn_silu1(x[base + e], mean, rstd, gamma[cc], beta[cc], sso, s1, sh1);
        }
        return;
    }
    const float ga = gamma[c], be = beta[c];
    const float sc1 = sso ? ss[(size_t)b * 2 * C + c] + 1.0f : 0.0f, sh = sso ? ss[(size_t)b * 2 * C + C + c] : 0.0f;
    const float *px = x + ((size_t)b * C + c) * HW;
    float *py = y + ((size_t)b * C + c) * HW;
    if ((HW & 3) == 0) {
        const int i = (ch * 256 + (int)threadIdx.x) * 4;
        if (i < HW) {
            float4 v = *reinterpret_cast<const float4 *>(px + i);
            v.x = gn_silu1(v.x, mean, rstd, ga, be, sso, sc1, sh);
            v.y = gn_silu1(v.y, mean, rstd, ga, be, sso, sc1, sh);
            v.z = gn_silu1(v.z, mean, rstd, ga, be, sso, sc1, sh);
            v.w = gn_silu1(v.w, mean, rstd, ga, be, sso, sc1, sh);
            *reinterpret_cast<float4 *>(py + i) = v;
        }
    } else {
        const int e1 = min(HW, (ch + 1) * 1024);
        for (int i = ch * 1024 + (int)threadIdx.x; i < e1; i += 256) py[i] = gn_silu1(px[i], mean, rstd, ga, be, sso, sc1, sh);
    }
}

// the same pass on statistics accumulated by the producing conv (k_conv_cc, a.gnp): wave 0 of each
// workgroup sums its (sample, group)'s per-tile partials — lane l takes tiles l, l+64, ... of the
// sample in order, then a fixed xor tree — and the pass adds an optional residual after the SiLU
// (ResnetBlock's identity shortcut, diffusion.py:168).  V float4 per thread (large batches: V = 4, so
// the per-workgroup statistics reduction is paid once per 4096 elements instead of 1024)
template <bool SMALL, int V = 1, typename TX = float>
__global__ __launch_bounds__(256) void k_gn_apply_t(int C, int HW, int G, int nch, const TX *__restrict__ x,
                                                    const float *__restrict__ gamma, const float *__restrict__ beta,
                                                    const float *__restrict__ ss, const double *__restrict__ gnp,
                                                    float eps, const float *__restrict__ post, float *__restrict__ y,
                                                    int bm = CC_BM)
{
    const int bg = blockIdx.y, b = bg / G, g = bg - b * G, cpg = C / G;
    const int cl = SMALL ? 0 : blockIdx.x / nch, ch = SMALL ? 0 : blockIdx.x - cl * nch;
    const int c = g * cpg + cl;
    const size_t base = ((size_t)b * C + c) * HW;
    // this thread's elements, residual and channel constants are loaded first (independent of the
    // statistics), so the statistics reduction below overlaps their latency
    const bool vec = (HW & 3) == 0;
    float4 v[V], r[V];
#pragma unroll
    for (int k = 0; k < V; ++k) {
        const int i4 = ((ch * V + k) * 256 + (int)threadIdx.x) * 4;
        v[k] = r[k] = float4{0.0f, 0.0f, 0.0f, 0.0f};
        if (!SMALL && vec && i4 < HW) {
            v[k] = ldx4(x + base + i4);
            if (post) r[k] = *reinterpret_cast<const float4 *>(post + base + i4);
        }
    }
    const float ga = gamma[c], be = beta[c];
    const bool sso = ss != nullptr;
    const float sc1 = sso ? ss[(size_t)b * 2 * C + c] + 1.0f : 0.0f, sh = sso ? ss[(size_t)b * 2 * C + C + c] : 0.0f;
    __shared__ float st2[2];
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        const int mlo = (int)(((int64_t)b * HW) / bm), mhi = (int)(((int64_t)(b + 1) * HW - 1) / bm);
        double s = 0.0, q = 0.0;
        for (int mt = mlo + lane; mt <= mhi; mt += 64) {
            const int slot = (int)(((int64_t)mt * bm) / HW) == b ? 0 : 1;
            const double *p = gnp + (((size_t)mt * G + g) * 2 + slot) * 2;
            s += p[0];
            q += p[1];
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            s += __shfl_xor(s, o, 64);
            q += __shfl_xor(q, o, 64);
        }
        if (lane == 0) {
            const double n = (double)cpg * HW, mean = s / n;
            double var = q / n - mean * mean;
            var = var < 0.0 ? 0.0 : var;
            st2[0] = (float)mean;
            st2[1] = (float)(1.0 / sqrt(var + (double)eps));
        }
    }
    __syncthreads();
    const float mean = st2[0], rstd = st2[1];
    if constexpr (SMALL) {        // small images: -nch whole channels of the group per workgroup
        const int cpb = -nch, cl0 = blockIdx.x * cpb, n = min(cpb, cpg - cl0) * HW;
        const size_t base0 = ((size_t)b * C + g * cpg + cl0) * HW;
        for (int e = threadIdx.x; e < n; e += 256) {
            const int cc = g * cpg + cl0 + e / HW;
            const float s1 = sso ? ss[(size_t)b * 2 * C + cc] + 1.0f : 0.0f, sh1 = sso ? ss[(size_t)b * 2 * C + C + cc] : 0.0f;
            float u = gn_silu1(ldx(x + base0 + e), mean, rstd, gamma[cc], beta[cc], sso, s1, sh1);
            if (post) u += post[base0 + e];
            y[base0 + e] = u;
        }
        return;
    }
    if (vec) {
#pragma unroll
        for (int k = 0; k < V; ++k) {
            const int i4 = ((ch * V + k) * 256 + (int)threadIdx.x) * 4;
            if (i4 < HW) {
                float4 u = v[k];
                u.x = gn_silu1(u.x, mean, rstd, ga, be, sso, sc1, sh);
                u.y = gn_silu1(u.y, mean, rstd, ga, be, sso, sc1, sh);
                u.z = gn_silu1(u.z, mean, rstd, ga, be, sso, sc1, sh);
                u.w = gn_silu1(u.w, mean, rstd, ga, be, sso, sc1, sh);
                if (post) { u.x += r[k].x; u.y += r[k].y; u.z += r[k].z; u.w += r[k].w; }
                *reinterpret_cast<float4 *>(y + base + i4) = u;
            }
        }
    } else {
        const int e1 = min(HW, (ch + 1) * 1024 * V);
        for (int i = ch * 1024 * V + (int)threadIdx.x; i < e1; i += 256) {
            float u = gn_silu1(ldx(x + base + i), mean, rstd, ga, be, sso, sc1, sh);
            if (post) u += post[base + i];
            y[base + i] = u;
        }
    }
}

// k_gn_apply_t's pass for a Block whose output feeds ONLY the next 3x3 bf16 conv (ResnetBlock's block1,
// diffusion.py:166-167): the same per-element arithmetic (statistics from the conv's per-tile
// partials, GN -> scale / shift -> SiLU), rounded to bf16 and stored as channel octets
// [B][C / 8][HW][8], the layout k_conv3_bf16<.., IN8> gathers with one 16-byte load per pixel.  The
// consumer rounds its operands to bf16 anyway, so its result is bit-identical to the fp32 path's
// while this pass writes half the bytes and the conv reads half.  Workgroup: 256 pixels of one
// (sample, group), every octet of the group.
template <typename TX = float>
__global__ __launch_bounds__(256) void k_gn_apply8(int C, int HW, int G, const TX *__restrict__ x,
                                                   const float *__restrict__ gamma, const float *__restrict__ beta,
                                                   const float *__restrict__ ss, const double *__restrict__ gnp,
                                                   float eps, __bf16 *__restrict__ y, int bm)
{
    const int bg = blockIdx.y, b = bg / G, g = bg - b * G, cpg = C / G;
    const int p = blockIdx.x * 256 + (int)threadIdx.x;
    __shared__ float st2[2];
    if (threadIdx.x < 64) {                     // (sample, group) statistics: k_gn_apply_t's reduction
        const int lane = threadIdx.x;
        const int mlo = (int)(((int64_t)b * HW) / bm), mhi = (int)(((int64_t)(b + 1) * HW - 1) / bm);
        double s = 0.0, q = 0.0;
        for (int mt = mlo + lane; mt <= mhi; mt += 64) {
            const int slot = (int)(((int64_t)mt * bm) / HW) == b ? 0 : 1;
            const double *pp = gnp + (((size_t)mt * G + g) * 2 + slot) * 2;
            s += pp[0];
            q += pp[1];
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            s += __shfl_xor(s, o, 64);
            q += __shfl_xor(q, o, 64);
        }
        if (lane == 0) {
            const double n = (double)cpg * HW, mean = s / n;
            double var = q / n - mean * mean;
            var = var < 0.0 ? 0.0 : var;
            st2[0] = (float)mean;
            st2[1] = (float)(1.0 / sqrt(var + (double)eps));
        }
    }
    // this thread's first octet in flight behind the statistics
    const int pc = min(p, HW - 1);
    const TX *xb = x + ((size_t)b * C + g * cpg) * HW + pc;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = ldx(xb + (size_t)j * HW);
    __syncthreads();
    const float mean = st2[0], rstd = st2[1];
    const bool sso = ss != nullptr;
    for (int o = 0; o < cpg / 8; ++o) {
        float nx[8];
        if (o + 1 < cpg / 8) {
#pragma unroll
            for (int j = 0; j < 8; ++j) nx[j] = ldx(xb + (size_t)(8 * (o + 1) + j) * HW);
        }
        bf16x8 h;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int c = g * cpg + 8 * o + j;
            const float sc1 = sso ? ss[(size_t)b * 2 * C + c] + 1.0f : 0.0f, sh = sso ? ss[(size_t)b * 2 * C + C + c] : 0.0f;
            h[j] = (__bf16)gn_silu1(v[j], mean, rstd, gamma[c], beta[c], sso, sc1, sh);
        }
        if (p < HW) *reinterpret_cast<bf16x8 *>(y + (((size_t)b * (C >> 3) + (g * cpg >> 3) + o) * HW + p) * 8) = h;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = nx[j];
    }
}

// k_gn_apply8 on the bf16 conv output with two adjacent pixels per thread (even HW): one 4-byte load per
// channel and 32 contiguous output bytes per thread instead of 2-byte loads and one 16-byte store;
// per element the same arithmetic, so the octets are k_gn_apply8's bit for bit.
__device__ __forceinline__ float2 ldx2(const __bf16 *p)
{
    const unsigned u = *reinterpret_cast<const unsigned *>(p);
    return float2{__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
}
__global__ __launch_bounds__(256) void k_gn_apply8x2(int C, int HW, int G, const __bf16 *__restrict__ x,
                                                     const float *__restrict__ gamma, const float *__restrict__ beta,
                                                     const float *__restrict__ ss, const double *__restrict__ gnp,
                                                     float eps, __bf16 *__restrict__ y, int bm)
{
    const int bg = blockIdx.y, b = bg / G, g = bg - b * G, cpg = C / G;
    const int p = (blockIdx.x * 256 + (int)threadIdx.x) * 2;   // HW even: p + 1 < HW whenever p < HW
    __shared__ float st2[2];
    if (threadIdx.x < 64) {                     // (sample, group) statistics: k_gn_apply_t's reduction
        const int lane = threadIdx.x;
        const int mlo = (int)(((int64_t)b * HW) / bm), mhi = (int)(((int64_t)(b + 1) * HW - 1) / bm);
        double s = 0.0, q = 0.0;
        for (int mt = mlo + lane; mt <= mhi; mt += 64) {
            const int slot = (int)(((int64_t)mt * bm) / HW) == b ? 0 : 1;
            const double *pp = gnp + (((size_t)mt * G + g) * 2 + slot) * 2;
            s += pp[0];
            q += pp[1];
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            s += __shfl_xor(s, o, 64);
            q += __shfl_xor(q, o, 64);
        }
        if (lane == 0) {
            const double n = (double)cpg * HW, mean = s / n;
            double var = q / n - mean * mean;
            var = var < 0.0 ? 0.0 : var;
            st2[0] = (float)mean;
            st2[1] = (float)(1.0 / sqrt(var + (double)eps));
        }
    }
    const int pc = min(p, HW - 2);
    const __bf16 *xb = x + ((size_t)b * C + g * cpg) * HW + pc;
    float2 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = ldx2(xb + (size_t)j * HW);
    __syncthreads();
    const float mean = st2[0], rstd = st2[1];
    const bool sso = ss != nullptr;
    for (int o = 0; o < cpg / 8; ++o) {
        float2 nx[8];
        if (o + 1 < cpg / 8) {
#pragma unroll
            for (int j = 0; j < 8; ++j) nx[j] = ldx2(xb + (size_t)(8 * (o + 1) + j) * HW);
        }
        bf16x8 h0, h1;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int c = g * cpg + 8 * o + j;
            const float sc1 = sso ? ss[(size_t)b * 2 * C + c] + 1.0f : 0.0f, sh = sso ? ss[(size_t)b * 2 * C + C + c] : 0.0f;
            h0[j] = (__bf16)gn_silu1(v[j].x, mean, rstd, gamma[c], beta[c], sso, sc1, sh);
            h1[j] = (__bf16)gn_silu1(v[j].y, mean, rstd, gamma[c], beta[c], sso, sc1, sh);
        }
        if (p < HW) {
            bf16x8 *yo = reinterpret_cast<bf16x8 *>(y + (((size_t)b * (C >> 3) + (g * cpg >> 3) + o) * HW + p) * 8);
            yo[0] = h0;
            yo[1] = h1;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = nx[j];
    }
}

// The U-Net's last two steps in one pass (diffusion.py:299-301): final_res_block's block2
// normalise pass (k_gn_apply_t's arithmetic: statistics from the conv's per-tile partials, GN ->
// scale/shift -> SiLU, + the res_conv shortcut) feeding final_conv, a 1x1 conv to NF <= 4 channels,
// without writing the C-channel activation.  Workgroup = 64 pixels of one sample, 16 waves; wave w takes
// channels [w C/16, (w+1) C/16) and the 1x1 sums are combined over the waves in wave order.
constexpr int GO_MAXF = 4, GO_NW = 16;
template <typename TX = float>
__global__ __launch_bounds__(64 * GO_NW) void k_gn_apply_out(int C, int HW, int G, const TX *__restrict__ x,
                                                             const float *__restrict__ gamma,
                                                             const float *__restrict__ beta,
                                                             const float *__restrict__ ss,
                                                             const double *__restrict__ gnp, float eps,
                                                             const float *__restrict__ post, int NF,
                                                             const float *__restrict__ wf,
                                                             const float *__restrict__ bf, float *__restrict__ yf,
                                                             int bm = CC_BM)
{
    __shared__ float st[64][2];
    __shared__ float part[GO_NW][GO_MAXF][64];
    const int b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int p = blockIdx.x * 64 + lane, cpg = C / G;
    const int cpw = (C + GO_NW - 1) / GO_NW, c0 = wv * cpw, c1 = min(C, c0 + cpw);
    const bool pv = p < HW;
    const int pc = pv ? p : HW - 1;
    // this lane's elements and shortcut values first: their loads overlap the statistics below
    float xv[4], rv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int c = min(c0 + u, C - 1);
        const size_t o = ((size_t)b * C + c) * HW + pc;
        xv[u] = ldx(x + o);
        rv[u] = post ? post[o] : 0.0f;
    }
    // (sample, group) statistics: wave w reduces groups w, w + GO_NW, ... exactly as k_gn_apply_t's wave 0
    for (int g = wv; g < G; g += GO_NW) {
        const int mlo = (int)(((int64_t)b * HW) / bm), mhi = (int)(((int64_t)(b + 1) * HW - 1) / bm);
        double s = 0.0, q = 0.0;
        for (int mt = mlo + lane; mt <= mhi; mt += 64) {
            const int slot = (int)(((int64_t)mt * bm) / HW) == b ? 0 : 1;
            const double *pp = gnp + (((size_t)mt * G + g) * 2 + slot) * 2;
            s += pp[0];
            q += pp[1];
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            s += __shfl_xor(s, o, 64);
            q += __shfl_xor(q, o, 64);
        }
        if (lane == 0) {
            const double n = (double)cpg * HW, mean = s / n;
            double var = q / n - mean * mean;
            var = var < 0.0 ? 0.0 : var;
            st[g][0] = (float)mean;
            st[g][1] = (float)(1.0 / sqrt(var + (double)eps));
        }
    }
    __syncthreads();
    float acc[GO_MAXF] = {0.0f, 0.0f, 0.0f, 0.0f};
    const bool sso = ss != nullptr;
    for (int c = c0; c < c1; ++c) {
        const int u = c - c0, g = c / cpg;
        const float xe = u < 4 ? xv[u] : ldx(x + ((size_t)b * C + c) * HW + pc);
        const float re = u < 4 ? rv[u] : (post ? post[((size_t)b * C + c) * HW + pc] : 0.0f);
        const float sc1 = sso ? ss[(size_t)b * 2 * C + c] + 1.0f : 0.0f, sh = sso ? ss[(size_t)b * 2 * C + C + c] : 0.0f;
        float v = gn_silu1(xe, st[g][0], st[g][1], gamma[c], beta[c], sso, sc1, sh);
        if (post) v += re;
#pragma unroll
        for (int f = 0; f < GO_MAXF; ++f)
            if (f < NF) acc[f] += wf[(size_t)f * C + c] * v;
    }
#pragma unroll
    for (int f = 0; f < GO_MAXF; ++f)
        if (f < NF) part[wv][f][lane] = acc[f];
    __syncthreads();
    if (wv == 0 && pv) {
        for (int f = 0; f < NF; ++f) {
            float v = part[0][f][lane];
            for (int w = 1; w < GO_NW; ++w) v += part[w][f][lane];
            yf[((size_t)b * NF + f) * HW + p] = v + (bf ? bf[f] : 0.0f);
        }
    }
}

// ----------------------------------------------------------------------------------- rmsnorm
// 64 pixels (lanes, coalesced) x 16 channel groups (waves) per workgroup: the channel sum of squares
// is split over the waves and combined in LDS in a fixed order, so small-HW stages (9x9 x 512
// channels) still spread over many lanes.
constexpr int RMS_G = 16;
__global__ __launch_bounds__(64 * RMS_G) void k_rmsnorm(int C, int HW, const float *__restrict__ x,
                                                        const float *__restrict__ g, const float *__restrict__ res,
                                                        float *__restrict__ y)
{
    __shared__ float part[RMS_G][64];
    const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
    const int pix = blockIdx.x * 64 + lane, b = blockIdx.y;
    const bool ok = pix < HW;
    const float *px = x + (size_t)b * C * HW + pix;
    float ssum = 0.0f;
    if (ok)
        for (int c = grp; c < C; c += RMS_G) { const float v = px[(size_t)c * HW]; ssum += v * v; }
    part[grp][lane] = ssum;
    __syncthreads();
    float tot = 0.0f;
#pragma unroll
    for (int i = 0; i < RMS_G; ++i) tot += part[i][lane];
    if (!ok) return;
    const float den = fmaxf(sqrtf(tot), 1e-12f);      // F.normalize: x / max(||x||, eps)
    const float sc = sqrtf((float)C);
    float *py = y + (size_t)b * C * HW + pix;
    const float *pr = res ? res + (size_t)b * C * HW + pix : nullptr;
    for (int c = grp; c < C; c += RMS_G) {
        float v = px[(size_t)c * HW] / den;
        v = v * g[c];
        v = v * sc;
        if (pr) v = v + pr[(size_t)c * HW];
        py[(size_t)c * HW] = v;
    }
}

// the same with the thread's NPT = ceil(C / G) channels held in registers between the two passes
// (one HBM read of x), loads issued together at clamped indices (no per-element branch), the
// residual loaded before the first store.  Workgroup = PX pixels x G = 1024 / PX channel groups:
// small images (the 9x9 / 18x18 levels) take narrow pixel blocks so that more than a couple of
// workgroups share the work and NPT stays small
template <int NPT, int PX>
__global__ __launch_bounds__(1024) void k_rmsnorm_r(int C, int HW, const float *__restrict__ x,
                                                    const float *__restrict__ g, const float *__restrict__ res,
                                                    float *__restrict__ y)
{
    constexpr int G = 1024 / PX;
    __shared__ float part[G][PX];
    const int lane = threadIdx.x % PX, grp = threadIdx.x / PX;
    const int pix = blockIdx.x * PX + lane, b = blockIdx.y;
    const bool ok = pix < HW;
    const size_t base = (size_t)b * C * HW + min(pix, HW - 1);
    float v[NPT];
#pragma unroll
    for (int i = 0; i < NPT; ++i) v[i] = x[base + (size_t)min(grp + i * G, C - 1) * HW];
    float ssum = 0.0f;
#pragma unroll
    for (int i = 0; i < NPT; ++i)
        if (grp + i * G < C) ssum += v[i] * v[i];
    part[grp][lane] = ssum;
    __syncthreads();
    float tot = 0.0f;
#pragma unroll 8
    for (int i = 0; i < G; ++i) tot += part[i][lane];
    float r[NPT] = {};
    if (res) {
#pragma unroll
        for (int i = 0; i < NPT; ++i) r[i] = res[base + (size_t)min(grp + i * G, C - 1) * HW];
    }
    if (!ok) return;
    const float den = fmaxf(sqrtf(tot), 1e-12f);      // F.normalize: x / max(||x||, eps)
    const float sc = sqrtf((float)C);
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
        const int c = grp + i * G;
        if (c >= C) break;
        float o = v[i] / den;
        o = o * g[c];
        o = o * sc;
        if (res) o = o + r[i];
        y[base + (size_t)c * HW] = o;
    }
}

template <int PX>
bool launch_rmsnorm_r(int B, int C, int HW, const float *x, const float *g, const float *res, float *y, hipStream_t st)
{
    constexpr int G = 1024 / PX;
    const dim3 grid((HW + PX - 1) / PX, B), blk(1024);
    if (C <= 2 * G) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_rmsnorm_r<2, PX>), grid, blk, 0, st, C, HW, x, g, res, y);
    else if (C <= 4 * G) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_rmsnorm_r<4, PX>), grid, blk, 0, st, C, HW, x, g, res, y);
    else if (C <= 8 * G) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_rmsnorm_r<8, PX>), grid, blk, 0, st, C, HW, x, g, res, y);
    else if (C <= 16 * G) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_rmsnorm_r<16, PX>), grid, blk, 0, st, C, HW, x, g, res, y);
    else return false;
    return true;
}

// ------------------------------------------------------------------------------------ linear
__global__ __launch_bounds__(256) void k_linear(int in, int out, const float *__restrict__ x,
                                                const float *__restrict__ w, const float *__restrict__ bias,
                                                int act_in, int act_out, float *__restrict__ y)
{
    const int o = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6), b = blockIdx.y, lane = threadIdx.x & 63;
    if (o >= out) return;
    const float *xb = x + (size_t)b * in;
    const float *wo = w + (size_t)o * in;
    float s = 0.0f;
    for (int i = lane; i < in; i += 64) {
        float v = xb[i];
        if (act_in == 1) v = v / (1.0f + expf(-v));
        s += wo[i] * v;
    }
    for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
    if (lane == 0) {
        float v = s + (bias ? bias[o] : 0.0f);
        if (act_out == 1) v = 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));   // nn.GELU (erf)
        y[(size_t)b * out + o] = v;
    }
}

__global__ void k_sinusoidal(int dim, float neg_emb, const int64_t *__restrict__ t, float *__restrict__ y)
{
    const int i = threadIdx.x, b = blockIdx.x, half = dim / 2;
    if (i >= half) return;
    const float f = expf((float)i * neg_emb);
    const float arg = (float)t[b] * f;
    y[(size_t)b * dim + i] = sinf(arg);
    y[(size_t)b * dim + half + i] = cosf(arg);
}

// Unet.time_mlp in one launch: SinusoidalPosEmb -> Linear -> GELU -> Linear.  Workgroup (row block,
// sample): every workgroup forms the embedding and the whole hidden layer (a thread per hidden row,
// its weight row loaded as float4s), then four output rows (a wave each)
constexpr int TM_ROWS = 4;
// the weight loads of 256 inputs are issued together (a dependent chain of loads would pay the
// memory latency once per 64 inputs); products accumulated in input order as in k_linear
__device__ __forceinline__ float wave_dot(const float *__restrict__ w, const float *x, int in, int lane, bool silu)
{
    float s = 0.0f;
    for (int i0 = 0; i0 < in; i0 += 256) {
        float wv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) wv[u] = w[min(i0 + lane + 64 * u, in - 1)];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = i0 + lane + 64 * u;
            if (i < in) {
                float v = x[i];
                if (silu) v = v / (1.0f + expf(-v));
                s += wv[u] * v;
            }
        }
    }
    for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
    return s;
}
struct TmArgs {
    int dim, hid, out;
    float neg_emb;
    const int64_t *t;
    const float *w1, *b1, *w2, *b2;
    float *y;
};
// row block bx of sample b; sm: dim + hid floats
__device__ __forceinline__ void time_mlp_rows(const TmArgs &m, int bx, int b, float *sm)
{
    const int dim = m.dim, hid = m.hid, out = m.out;
    const float neg_emb = m.neg_emb;
    const int64_t *__restrict__ t = m.t;
    const float *__restrict__ w1 = m.w1, *__restrict__ b1 = m.b1, *__restrict__ w2 = m.w2, *__restrict__ b2 = m.b2;
    float *__restrict__ y = m.y;
    float *e = sm, *h = sm + dim;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int half = dim / 2;
    for (int i = tid; i < half; i += 256) {
        const float f = expf((float)i * neg_emb);
        const float arg = (float)t[b] * f;
        e[i] = sinf(arg);
        e[half + i] = cosf(arg);
    }
    __syncthreads();
    for (int o = tid; o < hid; o += 256) {
        const float *wr = w1 + (size_t)o * dim;
        float s = 0.0f;
        if ((dim & 3) == 0) {
            for (int i = 0; i < dim; i += 4) {
                const float4 w4 = *reinterpret_cast<const float4 *>(wr + i);
                s += w4.x * e[i];
                s += w4.y * e[i + 1];
                s += w4.z * e[i + 2];
                s += w4.w * e[i + 3];
            }
        } else {
            for (int i = 0; i < dim; ++i) s += wr[i] * e[i];
        }
        const float v = s + b1[o];
        h[o] = 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));
    }
    __syncthreads();
    const int o = bx * TM_ROWS + wv;
    if (o >= out) return;
    const float s = wave_dot(w2 + (size_t)o * hid, h, hid, lane, false);
    if (lane == 0) y[(size_t)b * out + o] = s + b2[o];
}
__global__ __launch_bounds__(256) void k_time_mlp(TmArgs m)
{
    extern __shared__ float tm_sm[];
    time_mlp_rows(m, blockIdx.x, blockIdx.y, tm_sm);
}

// Large batches (the configs[4] tile batch, hundreds of samples): the time MLP for TMB samples per
// workgroup, so the hidden layer's weights are read once per sample block instead of once per
// (row block, sample); per sample the arithmetic is time_mlp_rows' (bit for bit k_time_mlp's).
constexpr int TMB = 8;
constexpr int TMB_RW = 8;                             // k_time_mlp_b: second-layer rows per wave
__global__ __launch_bounds__(256) void k_time_mlp_b(TmArgs m, int B)
{
    extern __shared__ float tmb_sm[];                 // [TMB][dim + hid]
    const int dim = m.dim, hid = m.hid, out = m.out, ld = dim + hid;
    const int b0 = blockIdx.y * TMB, nb = min(TMB, B - b0);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, half = dim / 2;
    for (int idx = tid; idx < nb * half; idx += 256) {
        const int bb = idx / half, i = idx - bb * half;
        const float f = expf((float)i * m.neg_emb);
        const float arg = (float)m.t[b0 + bb] * f;
        tmb_sm[bb * ld + i] = sinf(arg);
        tmb_sm[bb * ld + half + i] = cosf(arg);
    }
    __syncthreads();
    for (int o = tid; o < hid; o += 256) {
        const float *wr = m.w1 + (size_t)o * dim;
        for (int bb = 0; bb < nb; ++bb) {
            const float *e = tmb_sm + bb * ld;
            float s = 0.0f;
            if ((dim & 3) == 0) {
                for (int i = 0; i < dim; i += 4) {
                    const float4 w4 = *reinterpret_cast<const float4 *>(wr + i);
                    s += w4.x * e[i];
                    s += w4.y * e[i + 1];
                    s += w4.z * e[i + 2];
                    s += w4.w * e[i + 3];
                }
            } else {
                for (int i = 0; i < dim; ++i) s += wr[i] * e[i];
            }
            const float v = s + m.b1[o];
            tmb_sm[bb * ld + dim + o] = 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));
        }
    }
    __syncthreads();
    // second layer: TMB_RW rows per wave (the first layer above is formed once per block for them all,
    // not once per 4 rows: 311 -> a few us at 344 samples); per sample wave_dot's arithmetic
    for (int r = 0; r < TMB_RW; ++r) {
        const int o = (blockIdx.x * 4 + wv) * TMB_RW + r;
        if (o >= out) return;                         // wave-uniform
        for (int bb = 0; bb < nb; ++bb) {
            const float s = wave_dot(m.w2 + (size_t)o * hid, tmb_sm + bb * ld + dim, hid, lane, false);
            if (lane == 0) m.y[(size_t)(b0 + bb) * out + o] = s + m.b2[o];
        }
    }
}

// every ResnetBlock's time MLP, Linear(SiLU(t)) (diffusion.py:157-165), in one launch: up to
// LM_MAX linears sharing the input, one wave per output row
constexpr int LM_MAX = 32;
struct LinMulti {
    const float *w[LM_MAX];
    const float *b[LM_MAX];
    float *y[LM_MAX];
    int out[LM_MAX];
    int start[LM_MAX + 1];
    int n;
};
// LSM_RPW rows of the multi-linear per wave, their weight loads issued together; each row's
// arithmetic is wave_dot's (same order: k_linear_silu_multi's results bit for bit).  Workgroup blk
// of sample b: rows [blk * 4 * LSM_RPW, (blk + 1) * 4 * LSM_RPW).  Used as a side job of the
// first ResnetBlock's conv launch (k_conv_cc_lsm).
constexpr int LSM_RPW = 8;
template <int RPW>
__device__ __forceinline__ void lsm_rows(int in, const float *__restrict__ x, const LinMulti &L, int blk, int b)
{
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int g0 = (blk * 4 + wv) * RPW, gend = L.start[L.n];
    if (g0 >= gend) return;
    const float *wr[RPW];
    float *yo[RPW];
    float bo[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        const int go = min(g0 + r, gend - 1);
        int j = 0;
        while (go >= L.start[j + 1]) ++j;
        const int o = go - L.start[j];
        wr[r] = L.w[j] + (size_t)o * in;
        yo[r] = g0 + r < gend ? L.y[j] + (size_t)b * L.out[j] + o : nullptr;
        bo[r] = L.b[j] ? L.b[j][o] : 0.0f;
    }
    const float *xb = x + (size_t)b * in;
    float s[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r) s[r] = 0.0f;
    for (int i0 = 0; i0 < in; i0 += 256) {
        float wv4[RPW][4];
#pragma unroll
        for (int r = 0; r < RPW; ++r)
#pragma unroll
            for (int u = 0; u < 4; ++u) wv4[r][u] = wr[r][min(i0 + lane + 64 * u, in - 1)];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = i0 + lane + 64 * u;
            if (i < in) {
                float v = xb[i];
                v = v / (1.0f + expf(-v));
#pragma unroll
                for (int r = 0; r < RPW; ++r) s[r] += wv4[r][u] * v;
            }
        }
    }
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        float v = s[r];
        for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
        if (lane == 0 && yo[r]) *yo[r] = v + bo[r];
    }
}

// Large batches: SiLU(x) of LSB samples formed once per workgroup into LDS, then each wave runs
// wave_dot's arithmetic (bit for bit k_linear_silu_multi's) for LSR rows x the LSB samples, its row's
// weights re-read from the cache instead of once per sample from the whole weight set.
constexpr int LSB = 32, LSR = 16;
__global__ __launch_bounds__(256) void k_linear_silu_multi_b(int in, int B, const float *__restrict__ x, LinMulti L)
{
    extern __shared__ float lsb_sm[];                 // [LSB][in], SiLU'd
    const int b0 = blockIdx.y * LSB, nb = min(LSB, B - b0);
    for (int idx = threadIdx.x; idx < nb * in; idx += 256) {
        float v = x[(size_t)b0 * in + idx];
        lsb_sm[idx] = v / (1.0f + expf(-v));
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, gend = L.start[L.n];
    for (int rr = 0; rr < LSR; ++rr) {
        const int go = (blockIdx.x * 4 + wv) * LSR + rr;
        if (go >= gend) return;
        int j = 0;
        while (go >= L.start[j + 1]) ++j;
        const int o = go - L.start[j];
        const float *w = L.w[j] + (size_t)o * in;
        const float bo = L.b[j] ? L.b[j][o] : 0.0f;
        float wv4[4];                                 // in <= 256 (host check): one chunk, loaded once
#pragma unroll
        for (int u = 0; u < 4; ++u) wv4[u] = w[min(lane + 64 * u, in - 1)];
        // four samples at a time: independent chains, their reductions interleaved
        for (int bb0 = 0; bb0 < nb; bb0 += 4) {
            float s[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float *xs = lsb_sm + min(bb0 + q, nb - 1) * in;
                s[q] = 0.0f;
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int i = lane + 64 * u;
                    if (i < in) s[q] += wv4[u] * xs[i];
                }
            }
            for (int off = 32; off > 0; off >>= 1)
#pragma unroll
                for (int q = 0; q < 4; ++q) s[q] += __shfl_down(s[q], off, 64);
            if (lane == 0)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (bb0 + q < nb) L.y[j][(size_t)(b0 + bb0 + q) * L.out[j] + o] = s[q] + bo;
        }
    }
}

// Large batches, in = 256 (the dim-64 U-Net's time embedding): the same per-sample arithmetic as
// wave_dot -- lane k's partial p[k] = sum over u of w[k + 64u] x[k + 64u] as an FMA chain in u, then the
// shfl_down tree over k (pairs 32 apart first, then 16, ..., 1) -- evaluated with one SAMPLE per
// lane instead of one sample per wave: the tree is evaluated depth-first in registers
// (wdot_tree), so no cross-lane instruction is needed.  Each sample's result is bit for bit
// k_linear_silu_multi's.  Workgroup: 64 samples (SiLU'd into LDS as [k][u], rows of 260 floats: a
// leaf's four x values are one conflict-free ds_read_b128, round 6) x 4 waves x WDR rows; the rows' weights in LDS as [row][k][u]
// (one broadcast read per leaf).
constexpr int WDR = 8;
// wave_dot's shfl_down tree as a recursion: F(o, l) = F(2o, l) + F(2o, l + o), F(64, l) = lane l's
// partial (an FMA chain over u of w[l + 64u] x[l + 64u]); the sample's result is F(1, 0).  Every index
// is a template constant; one row at a time (independent rows let the scheduler interleave whole
// trees and spill).
template <int O, int LX>
__device__ __forceinline__ float wdot_tree(const float *__restrict__ xrow, const float *__restrict__ wrow, float dep)
{
    if constexpr (O == 64) {
        // the leaf's LDS offset passes through an asm that consumes the previous leaf group's value:
        // its reads are issued after that group (the scheduler would otherwise lift all 64 leaves')
        int ox = LX;
        asm volatile("" : "+v"(ox) : "v"(dep));
        const f32x4 w4 = *reinterpret_cast<const f32x4 *>(wrow + 4 * ox);    // [k][u]: one broadcast read
        const f32x4 x4 = *reinterpret_cast<const f32x4 *>(xrow + 4 * ox);    // [k][u]: one read per lane
        float sacc = 0.0f;
#pragma unroll
        for (int u = 0; u < 4; ++u) sacc = fmaf(w4[u], x4[u], sacc);
        return sacc;
    } else {
        const float a = wdot_tree<2 * O, LX>(xrow, wrow, dep);
        // groups of four leaves issue their reads together; each group waits for the previous one
        const float b = wdot_tree<2 * O, LX + O>(xrow, wrow, O < 16 ? a : dep);
        return a + b;
    }
}

__global__ __launch_bounds__(256) void k_wdot_silu_b(int B, const float *__restrict__ x, LinMulti L)
{
    __shared__ __attribute__((aligned(16))) float xs[64][260];   // [sample][k][u] (x index k + 64u); 1040-B rows:
                                                                   // a lane's ds_read_b128 per leaf, conflict-free
    __shared__ __attribute__((aligned(16))) float wt[4][WDR][64][4];   // [wave][row][k][u]
    const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int b0 = blockIdx.y * 64, nb = min(64, B - b0), gend = L.start[L.n];
    // staging with 16 loads in flight per thread (a load per iteration would be a latency chain)
    const int g0 = (blockIdx.x * 4 + wv) * WDR;
    const float *wr[WDR];
#pragma unroll
    for (int r = 0; r < WDR; ++r) {
        const int go = min(g0 + r, gend - 1);
        int j = 0;
        while (go >= L.start[j + 1]) ++j;
        wr[r] = L.w[j] + (size_t)(go - L.start[j]) * 256;
    }
    {
        float wv4[WDR][4];
#pragma unroll
        for (int r = 0; r < WDR; ++r)
#pragma unroll
            for (int u = 0; u < 4; ++u) wv4[r][u] = wr[r][lane + 64 * u];
#pragma unroll
        for (int r = 0; r < WDR; ++r)
#pragma unroll
            for (int u = 0; u < 4; ++u) wt[wv][r][lane][u] = wv4[r][u];
    }
#pragma unroll 1
    for (int it = 0; it < 64; it += 16) {
        float v[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int idx = (it + q) * 256 + tid, bb = idx >> 8;
            v[q] = x[(size_t)(b0 + min(bb, nb - 1)) * 256 + (idx & 255)];
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int idx = (it + q) * 256 + tid;
            xs[idx >> 8][(idx & 63) * 4 + ((idx >> 6) & 3)] = v[q] / (1.0f + expf(-v[q]));
        }
    }
    __syncthreads();
    const int b = b0 + lane;
#pragma unroll 1
    for (int r = 0; r < WDR; ++r) {
        const int go = g0 + r;
        if (go >= gend) break;                      // wave-uniform
        const float res = wdot_tree<1, 0>(xs[lane], &wt[wv][r][0][0], 0.0f);
        int j = 0;
        while (go >= L.start[j + 1]) ++j;
        const int o = go - L.start[j];
        if (lane < nb) L.y[j][(size_t)b * L.out[j] + o] = res + (L.b[j] ? L.b[j][o] : 0.0f);
    }
}

__global__ __launch_bounds__(256) void k_linear_silu_multi(int in, const float *__restrict__ x, LinMulti L)
{
    const int go = blockIdx.x * 4 + (threadIdx.x >> 6), b = blockIdx.y, lane = threadIdx.x & 63;
    if (go >= L.start[L.n]) return;
    int j = 0;
    while (go >= L.start[j + 1]) ++j;
    const int o = go - L.start[j];
    const float s = wave_dot(L.w[j] + (size_t)o * in, x + (size_t)b * in, in, lane, true);
    if (lane == 0) L.y[j][(size_t)b * L.out[j] + o] = s + (L.b[j] ? L.b[j][o] : 0.0f);
}

// The U-Net's first launch (Unet.forward, diffusion.py:276-279): init_conv (k_conv_ig tiles,
// blockIdx.x < gxc; a single n tile, no K split) and the time MLP (the rest of the grid, as
// k_time_mlp) are independent, so they share one launch.  Each role's arithmetic is that of its
// own kernel, bit for bit.
template <int KH>
__global__ __launch_bounds__(256, 2) void k_unet_head(IgArgs a, int gxc, TmArgs m, int tm_x)
{
    __shared__ __attribute__((aligned(16))) float sm[IG_SMEM];
    const int bx = blockIdx.x;
    if (bx < gxc) {
        conv_ig_tile<KH, RDQ_IN_PLAIN>(a, bx, 0, 0, sm);
    } else {
        const int r = bx - gxc;
        time_mlp_rows(m, r % tm_x, r / tm_x, sm);
    }
}

// The first ResnetBlock's conv (GroupNorm statistics in its epilogue) with every ResnetBlock's
// Linear(SiLU(t)) as a side job: blockIdx.x < nlsm (y = z = 0) runs lsm_rows, the rest the conv tiles
// of k_conv_cc.  Measured at B = 1 (tools/lsm_ab.py): 1.7 us under the two separate launches — the
// side job's workgroups slow the conv about as much as their own launch costs, so the Python side
// uses this form for B <= 2 only.  The GroupNorm pass that follows reads this block's scale/shift.
template <int TAPS, int MODE>
__global__ __launch_bounds__(256, 2) void k_conv_cc_lsm(CcArgs a, LinMulti L, int in, const float *temb, int nlsm,
                                                        int lsm_per_b)
{
    __shared__ __attribute__((aligned(16))) float sm[CC_SMEM];
    const int bx = blockIdx.x;
    if (bx < nlsm) {
        if (blockIdx.y == 0 && blockIdx.z == 0) lsm_rows<LSM_RPW>(in, temb, L, bx % lsm_per_b, bx / lsm_per_b);
        return;
    }
    conv_cc_tile<TAPS, MODE, false>(a, bx - nlsm, blockIdx.y, blockIdx.z, gridDim.x - nlsm, gridDim.y, sm);
}

// -------------------------------------------------------------------------- linear attention
// k softmax over the (memory + pixel) tokens per (b, h, d) folded into the context (flash style): a
// chunk of LA_CH tokens forms exp(k - m_c) with its OWN row maxima m_c, the partial context
// sum_j exp(k[d][j] - m_c[d]) v[e][j] and the partial sum s_c[d]; the combine rescales the chunks
// by exp(m_c - max_c m_c) in chunk order.  No separate statistics pass over all tokens.
constexpr int LA_CH = 256;
__global__ __launch_bounds__(256) void k_la_ctx(int heads, int dh, int n, int nmem, const float *__restrict__ qkv,
                                                const float *__restrict__ mem, float *__restrict__ part,
                                                float *__restrict__ pstat)
{
    __shared__ float P[32][LA_CH + 1], V[32][LA_CH + 1];
    const int ch = blockIdx.x, h = blockIdx.y, b = blockIdx.z, tid = threadIdx.x;
    const int C = heads * dh, nk = nmem + n;
    const int j0 = ch * LA_CH;
    const float *kb = qkv + ((size_t)b * 3 * C + C + h * dh) * n;
    const float *vb = qkv + ((size_t)b * 3 * C + 2 * C + h * dh) * n;
    const float *mk = mem + (size_t)(0 * heads + h) * dh * nmem;
    const float *mv = mem + (size_t)(1 * heads + h) * dh * nmem;
    {
        // thread = token j0 + tid: its dh keys and values (stride n, or nmem for memory tokens)
        // loaded together, then staged as rows d of P and V
        const int j = j0 + tid;
        const bool in = j < nk, memtok = j < nmem;
        const float *kp = memtok ? mk + j : kb + (in ? j - nmem : 0);
        const float *vp = memtok ? mv + j : vb + (in ? j - nmem : 0);
        const int stride = memtok ? nmem : n;
        float kr[32], vr[32];
#pragma unroll
        for (int d = 0; d < 32; ++d) {
            const int dd = min(d, dh - 1);
            kr[d] = kp[(size_t)dd * stride];
            vr[d] = vp[(size_t)dd * stride];
        }
#pragma unroll
        for (int d = 0; d < 32; ++d)
            if (d < dh) {
                P[d][tid] = in ? kr[d] : -INFINITY;
                V[d][tid] = in ? vr[d] : 0.0f;                   // row d of V = value channel e = d
            }
    }
    __syncthreads();
    // row maxima and exp / sums: 8 threads per row d, 32 tokens each, fixed xor trees
    {
        const int d = tid >> 3, q = tid & 7;
        float m = -INFINITY;
        if (d < dh)
            for (int jj = q; jj < LA_CH; jj += 8) m = fmaxf(m, P[d][jj]);
#pragma unroll
        for (int o = 1; o < 8; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 8));
        float sm = 0.0f;
        if (d < dh)
            for (int jj = q; jj < LA_CH; jj += 8) {
                const float e = P[d][jj] == -INFINITY ? 0.0f : expf(P[d][jj] - m);
                P[d][jj] = e;
                sm += e;
            }
#pragma unroll
        for (int o = 1; o < 8; o <<= 1) sm += __shfl_xor(sm, o, 8);
        if (d < dh && q == 0) {
            float *ps = pstat + (((size_t)ch * gridDim.z + b) * heads + h) * dh * 2 + 2 * d;
            ps[0] = m;
            ps[1] = sm;
        }
    }
    __syncthreads();
    float *o = part + (((size_t)ch * gridDim.z + b) * heads + h) * dh * dh;
    if (dh == 32) {
        // ctx[d][e] = sum_j P[d][j] V[e][j] is a 32 x 32 GEMM with K = the chunk's tokens: each wave
        // takes 64 of them on v_mfma_f32_32x32x2_f32 (A[row l&31][k l>>5] = P, B[k l>>5][col l&31] = V),
        // then the four partial tiles are summed through LDS in a fixed order
        const int w = tid >> 6, l = tid & 63;
        f32x16 acc = {};
#pragma unroll 8
        for (int i = 0; i < LA_CH / 8; ++i) {
            const int jj = w * (LA_CH / 4) + 2 * i + (l >> 5);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(P[l & 31][jj], V[l & 31][jj], acc, 0, 0, 0);
        }
        __syncthreads();
        float *R = &P[0][0];                                     // 4 x 1024 floats (P holds 32 x 257)
#pragma unroll
        for (int r = 0; r < 16; ++r) R[w * 1024 + ((r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * 32 + (l & 31)] = acc[r];
        __syncthreads();
        for (int i = tid; i < 1024; i += 256) o[i] = ((R[i] + R[1024 + i]) + R[2048 + i]) + R[3072 + i];
        return;
    }
    // dh < 32: 256 threads x 4 outputs: (d, e) = (tid >> 3, (tid & 7) * 4 + q)
    const int d = tid >> 3, e0 = (tid & 7) * 4;
    if (d >= dh) return;
    float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    for (int jj = 0; jj < LA_CH; ++jj) {
        const float p = P[d][jj];
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] += p * V[e0 + q][jj];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) if (e0 + q < dh) o[(size_t)d * dh + e0 + q] = acc[q];
}

// ctx[b][h][d][e] = sum_c exp(m_c[d] - M[d]) part_c[d][e] / sum_c exp(m_c[d] - M[d]) s_c[d], chunks in
// order (M = the maximum over the chunks)
__global__ __launch_bounds__(256) void k_la_reduce(int BHDD, int dh, int nch, const float *__restrict__ pstat,
                                                   const float *__restrict__ part, float *__restrict__ ctx)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= BHDD) return;
    const int row = i / dh;                                      // (b, h, d)
    const int BHD = BHDD / dh;
    // chunk statistics and partials read in groups of 8 (loads in flight together), combined in order
    float M = -INFINITY;
    for (int c0 = 0; c0 < nch; c0 += 8) {
        float mv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) mv[u] = pstat[((size_t)min(c0 + u, nch - 1) * BHD + row) * 2];
#pragma unroll
        for (int u = 0; u < 8; ++u) M = fmaxf(M, mv[u]);
    }
    float num = 0.0f, den = 0.0f;
    for (int c0 = 0; c0 < nch; c0 += 8) {
        float mv[8], sv[8], pv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int c = min(c0 + u, nch - 1);
            mv[u] = pstat[((size_t)c * BHD + row) * 2];
            sv[u] = pstat[((size_t)c * BHD + row) * 2 + 1];
            pv[u] = part[(size_t)c * BHDD + i];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (c0 + u < nch) {
                const float f = expf(mv[u] - M);
                num += f * pv[u];
                den += f * sv[u];
            }
    }
    ctx[i] = num / den;
}

// per (b, h, pixel): q softmax over d, scale, out[e] = sum_d ctx[d][e] q[d].  Workgroup = 64 pixels
// x 4 quarters of the 32 output channels e (a thread forms the softmax of its pixel and 8 outputs)
__global__ __launch_bounds__(256) void k_la_out(int heads, int dh, int n, float scale,
                                                const float *__restrict__ qkv, const float *__restrict__ ctx,
                                                float *__restrict__ out)
{
    const int h = blockIdx.y, b = blockIdx.z;
    const int C = heads * dh;
    __shared__ __attribute__((aligned(16))) float cs[32][32];
    const float *cb = ctx + (size_t)(b * heads + h) * dh * dh;
    {
        float cv[4];                                             // dh * dh <= 1024: four loads in flight
#pragma unroll
        for (int u = 0; u < 4; ++u) cv[u] = cb[min(u * 256 + (int)threadIdx.x, dh * dh - 1)];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = u * 256 + (int)threadIdx.x;
            if (i < dh * dh) cs[i / dh][i % dh] = cv[u];
        }
    }
    __syncthreads();
    const int px = threadIdx.x & 63, eq = threadIdx.x >> 6;
    const int pix = blockIdx.x * 64 + px;
    if (pix >= n || eq * 8 >= dh) return;
    const float *q = qkv + ((size_t)b * 3 * C + h * dh) * n + pix;
    float qv[32];
    float mx = -INFINITY;
#pragma unroll
    for (int d = 0; d < 32; ++d) qv[d] = q[(size_t)min(d, dh - 1) * n];   // no branch per load
#pragma unroll
    for (int d = 0; d < 32; ++d) if (d < dh) mx = fmaxf(mx, qv[d]);
    float sm = 0.0f;
#pragma unroll
    for (int d = 0; d < 32; ++d) if (d < dh) { qv[d] = expf(qv[d] - mx); sm += qv[d]; }
#pragma unroll
    for (int d = 0; d < 32; ++d) if (d < dh) qv[d] = (qv[d] / sm) * scale;
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = 0.0f;
#pragma unroll
    for (int d = 0; d < 32; ++d) {
        if (d < dh) {
#pragma unroll
            for (int e4 = 0; e4 < 2; ++e4) {
                const f32x4 c4 = *reinterpret_cast<const f32x4 *>(&cs[d][eq * 8 + e4 * 4]);
#pragma unroll
                for (int q4 = 0; q4 < 4; ++q4) o[e4 * 4 + q4] += c4[q4] * qv[d];
            }
        }
    }
    float *ob = out + ((size_t)b * C + h * dh) * n + pix;
#pragma unroll
    for (int e = 0; e < 8; ++e) if (eq * 8 + e < dh) ob[(size_t)(eq * 8 + e) * n] = o[e];
}

// LinearAttention.forward from the partial contexts on: the chunk combine (k_la_reduce's order), the
// q softmax / context product (k_la_out's order), to_out = Conv2d(hidden, dim, 1) + bias, the to_out
// RMSNorm and the block's residual (diffusion.py:182-195, 286/297) in ONE launch.  Workgroup = PX
// pixels of one sample (PX = 32 at dim 64, else 16):
//   A  combine: per (h, d) row the chunk weights exp(m_c - M) and the denominator into LDS, then
//      ctx[h][d][e] = (sum_c f_c part_c) / den for all heads (nch = 0: ctx already combined in ws)
//   B  hidden[h*dh + e][p] = sum_d ctx[h][d][e] softmax_d(q)[d] * scale   (dh = 32)
//   C  y[o][p] = bias[o] + sum_c W[o][c] hidden[c][p] on v_mfma_f32_16x16x4_f32: wave w takes the
//      16-row o blocks w, w + 4, ..., the lane's W fragment (32 contiguous c of one row, k order
//      k = (lane >> 4) * 32 + step for W and hidden alike) loaded at the start of the launch so
//      its latency hides behind A and B
//   D  y / max(||y[:, p]||, 1e-12) * g * sqrt(dim) + x   (pixel-fastest stores)
// The fused form replaces k_la_reduce + k_la_out + the 1x1 conv + k_rmsnorm_r: four dependent
// launches of a few microseconds each at B = 1, where the launch is most of the cost.
constexpr int LAO_MAXCH = 8;                    // chunk partials combined in the launch up to this count
template <int DIM> struct LaoCfg { static constexpr int PX = DIM == 64 ? 32 : 16; };
template <int DIM>
__global__ __launch_bounds__(256) void k_la_out_proj(int heads, int n, int nch, float scale,
                                                     const float *__restrict__ qkv, const float *__restrict__ pstat,
                                                     const float *__restrict__ part, const float *__restrict__ w,
                                                     const float *__restrict__ bias, const float *__restrict__ g,
                                                     const float *__restrict__ res, float *__restrict__ y)
{
    constexpr int DH = 32, PX = LaoCfg<DIM>::PX, LDP = PX + 4, NG = 256 / PX, NR = DIM / NG;
    constexpr int NOB = DIM / 64, NPB = PX / 16, CH = 128;     // heads * DH = 128 (4 heads)
    extern __shared__ __attribute__((aligned(16))) float lo_sm[];
    const int HDD = CH * DH;
    float *cs = lo_sm;                          // [heads][DH][DH]
    float *hid = cs + HDD;                      // row r at r * PX + (r >> 5) * 16 (bank skew per head)
    float *ys = hid + CH * PX + 64;             // [DIM][LDP]
    float *red = ys + DIM * LDP;                // [NG][PX]
    float *tot = red + 256;                     // [PX]
    float *fst = tot + PX;                      // [nch][CH] chunk weights, then [CH] denominators
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, b = blockIdx.y, B = gridDim.y;
    const int px0 = blockIdx.x * PX;
    // the lane's W fragments: o block wv + 4 j, row (lane & 15), c = (lane >> 4) * 32 .. + 31
    f32x4 wf[NOB][8];
#pragma unroll
    for (int j = 0; j < NOB; ++j)
#pragma unroll
        for (int u = 0; u < 8; ++u)
            wf[j][u] = *reinterpret_cast<const f32x4 *>(w + (size_t)((wv + 4 * j) * 16 + (lane & 15)) * CH +
                                                        (lane >> 4) * 32 + u * 4);
    // residual (pixel-fastest: thread -> pixel tid % PX, channels tid / PX + k NG)
    const int ep = tid % PX, eg = tid / PX;
    const int epix = min(px0 + ep, n - 1);
    float rv[NR];
#pragma unroll
    for (int k = 0; k < NR; ++k) rv[k] = res ? res[((size_t)b * DIM + eg + k * NG) * n + epix] : 0.0f;
    // the first task's q column (phase B below) in flight behind the context combine
    const int ntask = PX * heads * 4;
    auto task_pix = [&](int t) { return px0 + t % PX; };
    auto load_q = [&](int t, float (&qv)[DH]) {
        const int h = t / (PX * 4);
        const float *q = qkv + ((size_t)b * 3 * CH + h * DH) * n + min(task_pix(t), n - 1);
#pragma unroll
        for (int d = 0; d < DH; ++d) qv[d] = q[(size_t)d * n];
    };
    float qv0[DH];
    load_q(tid, qv0);
    // A: combined context of every head
    if (nch > 0) {
        // nch <= LAO_MAXCH: every statistic of a row and a thread's partials are loaded together,
        // combined in chunk order as k_la_reduce does
        const int BHD = B * CH;
        if (tid < CH) {
            const int r = tid;
            const size_t row = (size_t)b * CH + r;
            float mv[LAO_MAXCH], sv[LAO_MAXCH];
#pragma unroll
            for (int c = 0; c < LAO_MAXCH; ++c) {
                const size_t k = ((size_t)min(c, nch - 1) * BHD + row) * 2;
                mv[c] = pstat[k];
                sv[c] = pstat[k + 1];
            }
            float M = -INFINITY;
#pragma unroll
            for (int c = 0; c < LAO_MAXCH; ++c) if (c < nch) M = fmaxf(M, mv[c]);
            float den = 0.0f;
#pragma unroll
            for (int c = 0; c < LAO_MAXCH; ++c)
                if (c < nch) {
                    const float f = expf(mv[c] - M);
                    fst[c * CH + r] = f;
                    den += f * sv[c];
                }
            fst[LAO_MAXCH * CH + r] = den;
        }
        const float *pb = part + (size_t)b * HDD;
        // this thread's 4 float4 entries (i4 = tid + 256 u) in two halves of 2 x LAO_MAXCH loads
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            f32x4 pv[2][LAO_MAXCH];
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int c = 0; c < LAO_MAXCH; ++c)
                    pv[u][c] = *reinterpret_cast<const f32x4 *>(pb + (size_t)min(c, nch - 1) * B * HDD +
                                                                (tid + 256 * (2 * hf + u)) * 4);
            if (hf == 0) __syncthreads();                          // fst complete
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int i4 = tid + 256 * (2 * hf + u), r = (i4 * 4) / DH;
                f32x4 num = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
                for (int c = 0; c < LAO_MAXCH; ++c)
                    if (c < nch) {
                        const float f = fst[c * CH + r];
#pragma unroll
                        for (int j = 0; j < 4; ++j) num[j] += f * pv[u][c][j];
                    }
                const float den = fst[LAO_MAXCH * CH + r];
#pragma unroll
                for (int j = 0; j < 4; ++j) cs[i4 * 4 + j] = num[j] / den;
            }
        }
    } else {
        const float *cb = part + (size_t)b * HDD;          // nch = 0: `part` is the combined context
        f32x4 cv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) cv[u] = *reinterpret_cast<const f32x4 *>(cb + (tid + 256 * u) * 4);
#pragma unroll
        for (int u = 0; u < 4; ++u) *reinterpret_cast<f32x4 *>(cs + (tid + 256 * u) * 4) = cv[u];
    }
    __syncthreads();
    // B: task (pixel, head, eighth eq) -> 8 hidden channels of one pixel
    for (int t = tid; t < ntask; t += 256) {
        const int p = t % PX, eq = (t / PX) & 3, h = t / (PX * 4);
        float qv[DH];
        if (t == tid) {
#pragma unroll
            for (int d = 0; d < DH; ++d) qv[d] = qv0[d];
        } else {
            load_q(t, qv);
        }
        float mx = -INFINITY;
#pragma unroll
        for (int d = 0; d < DH; ++d) mx = fmaxf(mx, qv[d]);
        float sm = 0.0f;
#pragma unroll
        for (int d = 0; d < DH; ++d) { qv[d] = expf(qv[d] - mx); sm += qv[d]; }
#pragma unroll
        for (int d = 0; d < DH; ++d) qv[d] = (qv[d] / sm) * scale;
        const float *ch = cs + h * DH * DH;
        float o[8] = {};
#pragma unroll
        for (int d = 0; d < DH; ++d) {
#pragma unroll
            for (int e4 = 0; e4 < 2; ++e4) {
                const f32x4 c4 = *reinterpret_cast<const f32x4 *>(&ch[d * DH + eq * 8 + e4 * 4]);
#pragma unroll
                for (int q4 = 0; q4 < 4; ++q4) o[e4 * 4 + q4] += c4[q4] * qv[d];
            }
        }
        const bool ok = px0 + p < n;
#pragma unroll
        for (int e = 0; e < 8; ++e) hid[(h * DH + eq * 8 + e) * PX + h * 16 + p] = ok ? o[e] : 0.0f;
    }
    __syncthreads();
    // C: MFMA projection
    {
        f32x4 acc[NOB][NPB];
#pragma unroll
        for (int j = 0; j < NOB; ++j)
#pragma unroll
            for (int pb = 0; pb < NPB; ++pb) acc[j][pb] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        const int kr = (lane >> 4) * 32;
        const float *hrow = hid + kr * PX + (lane >> 4) * 16 + (lane & 15);
#pragma unroll
        for (int s = 0; s < 32; ++s) {
            float bv[NPB];
#pragma unroll
            for (int pb = 0; pb < NPB; ++pb) bv[pb] = hrow[s * PX + pb * 16];
#pragma unroll
            for (int j = 0; j < NOB; ++j)
#pragma unroll
                for (int pb = 0; pb < NPB; ++pb)
                    acc[j][pb] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[j][s >> 2][s & 3], bv[pb], acc[j][pb], 0, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < NOB; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int o = (wv + 4 * j) * 16 + (lane >> 4) * 4 + r;
                const float bo = bias ? bias[o] : 0.0f;
#pragma unroll
                for (int pb = 0; pb < NPB; ++pb) ys[o * LDP + pb * 16 + (lane & 15)] = acc[j][pb][r] + bo;
            }
    }
    __syncthreads();
    // D: squared norms per pixel (channel groups, then the groups in order)
    {
        float s = 0.0f;
#pragma unroll
        for (int k = 0; k < NR; ++k) { const float v = ys[(eg + k * NG) * LDP + ep]; s += v * v; }
        red[eg * PX + ep] = s;
    }
    __syncthreads();
    if (tid < PX) {
        float s = 0.0f;
#pragma unroll
        for (int k = 0; k < NG; ++k) s += red[k * PX + tid];
        tot[tid] = s;
    }
    __syncthreads();
    if (px0 + ep >= n) return;
    const float den = fmaxf(sqrtf(tot[ep]), 1e-12f);          // F.normalize: x / max(||x||, eps)
    const float sc = sqrtf((float)DIM);
#pragma unroll
    for (int k = 0; k < NR; ++k) {
        const int o = eg + k * NG;
        float v = ys[o * LDP + ep] / den;
        v = v * g[o];
        v = v * sc;
        if (res) v = v + rv[k];
        y[((size_t)b * DIM + o) * n + px0 + ep] = v;
    }
}

template <int DIM>
static void launch_la_out_proj(int B, int heads, int n, int nch, float scale, const float *qkv, const float *pstat,
                               const float *part, const float *w, const float *bias, const float *g,
                               const float *res, float *y, hipStream_t st)
{
    constexpr int PX = LaoCfg<DIM>::PX;
    const size_t lds = ((size_t)128 * 32 + 128 * PX + 64 + (size_t)DIM * (PX + 4) + 256 + PX +
                        (size_t)(LAO_MAXCH + 1) * 128) * sizeof(float);
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_la_out_proj<DIM>), dim3((n + PX - 1) / PX, B), dim3(256), lds, st, heads, n,
                       nch, scale, qkv, pstat, part, w, bias, g, res, y);
}

// ---------------------------------------------------------------------------- full attention
// Workgroup = (b, h, 32 queries) x FA_KS key splits: thread (query i, split ks) runs an online
// softmax over the keys j = ks (mod FA_KS) from LDS; the FA_KS partial (max, sum, o[32]) of a query
// are merged in a fixed order, each split thread finishing 32 / FA_KS output channels.
constexpr int FA_KS = 8, FA_QB = 256 / FA_KS;
template <int DH>
__global__ __launch_bounds__(256) void k_full_attn(int heads, int n, int nmem, const float *__restrict__ qkv,
                                                   const float *__restrict__ mem, float *__restrict__ out)
{
    constexpr int dh = DH, LD = DH + 1;
    const int h = blockIdx.x, b = blockIdx.y;
    const int C = heads * dh, nk = nmem + n;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float *Ks = sm;                      // [nk][LD]
    float *Vs = Ks + nk * LD;            // [nk][LD]
    float *Po = Vs + nk * LD;            // [256][LD + 2]: o[0..dh), m, l per (query, split)
    const float *kb = qkv + ((size_t)b * 3 * C + C + h * dh) * n;
    const float *vb = qkv + ((size_t)b * 3 * C + 2 * C + h * dh) * n;
    // K / V of the head staged 8 elements per thread at a time (loads issued together)
    for (int i0 = 0; i0 < nk * dh; i0 += 8 * 256) {
        float kv[8], vv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = min(i0 + u * 256 + (int)threadIdx.x, nk * dh - 1);
            const int j = i / dh, d = i - j * dh;
            const float *kp = j < nmem ? mem + (((size_t)0 * heads + h) * nmem + j) * dh + d : kb + (size_t)d * n + (j - nmem);
            const float *vp = j < nmem ? mem + (((size_t)1 * heads + h) * nmem + j) * dh + d : vb + (size_t)d * n + (j - nmem);
            kv[u] = *kp;
            vv[u] = *vp;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = i0 + u * 256 + (int)threadIdx.x;
            if (i < nk * dh) {
                const int j = i / dh, d = i - j * dh;
                Ks[j * LD + d] = kv[u];
                Vs[j * LD + d] = vv[u];
            }
        }
    }
    __syncthreads();
    const int ql = threadIdx.x % FA_QB, ks = threadIdx.x / FA_QB;
    const int qi = blockIdx.z * FA_QB + ql;
    const bool qok = qi < n;
    float q[DH], o[DH];
    const float *qb = qkv + ((size_t)b * 3 * C + h * dh) * n + (qok ? qi : 0);
#pragma unroll
    for (int d = 0; d < dh; ++d) { q[d] = qok ? qb[(size_t)d * n] : 0.0f; o[d] = 0.0f; }
    const float scale = 1.0f / sqrtf((float)dh);
    float m = -INFINITY, l = 0.0f;
    for (int j = ks; j < nk; j += FA_KS) {
        float sc = 0.0f;
#pragma unroll
        for (int d = 0; d < dh; ++d) sc += q[d] * Ks[j * LD + d];
        sc = sc * scale;
        const float mn = fmaxf(m, sc);
        const float corr = expf(m - mn), p = expf(sc - mn);
        l = l * corr + p;
#pragma unroll
        for (int d = 0; d < dh; ++d) o[d] = o[d] * corr + p * Vs[j * LD + d];
        m = mn;
    }
    float *po = Po + (size_t)threadIdx.x * (LD + 2);
#pragma unroll
    for (int d = 0; d < dh; ++d) po[d] = o[d];
    po[LD] = m;
    po[LD + 1] = l;
    __syncthreads();
    if (!qok) return;
    // merge the FA_KS partials of query ql in split order; this thread writes channels ks*dh/FA_KS...
    float M = -INFINITY;
#pragma unroll
    for (int k2 = 0; k2 < FA_KS; ++k2) M = fmaxf(M, Po[(size_t)(k2 * FA_QB + ql) * (LD + 2) + LD]);
    float Lsum = 0.0f, w[FA_KS];
#pragma unroll
    for (int k2 = 0; k2 < FA_KS; ++k2) {
        const float *pk = Po + (size_t)(k2 * FA_QB + ql) * (LD + 2);
        w[k2] = pk[LD] == -INFINITY ? 0.0f : expf(pk[LD] - M);
        Lsum += pk[LD + 1] * w[k2];
    }
    constexpr int DPS = DH / FA_KS;
    float *ob = out + ((size_t)b * C + h * dh) * n + qi;
#pragma unroll
    for (int dd = 0; dd < DPS; ++dd) {
        const int d = ks * DPS + dd;
        float t = 0.0f;
#pragma unroll
        for (int k2 = 0; k2 < FA_KS; ++k2) t += Po[(size_t)(k2 * FA_QB + ql) * (LD + 2) + d] * w[k2];
        ob[(size_t)d * n] = t / Lsum;
    }
}

// -------------------------------------------------------------------------- RED elementwise
__global__ __launch_bounds__(256) void k_red_q_sample(int64_t n, const float *__restrict__ sa,
                                                      const float *__restrict__ s1a, const int64_t *__restrict__ t,
                                                      const float *__restrict__ x0, const float *__restrict__ eps,
                                                      float *__restrict__ xt, int64_t *__restrict__ t_out)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int b = blockIdx.y;
    if (i >= n) return;
    const int64_t tb = t[b];
    if (t_out && i == 0) t_out[b] = tb;
    const size_t o = (size_t)b * n + i;
    const float a1 = sa[tb] * x0[o];
    const float a2 = s1a[tb] * eps[o];
    xt[o] = a1 + a2;
}

__global__ __launch_bounds__(256) void k_red_epilogue(int64_t n, const float *__restrict__ sr,
                                                      const float *__restrict__ srm1, const int64_t *__restrict__ t,
                                                      const float *__restrict__ xt, const float *__restrict__ eh,
                                                      const float *__restrict__ eps, float *__restrict__ g)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int b = blockIdx.y;
    if (i >= n) return;
    const int64_t tb = t[b];
    const size_t o = (size_t)b * n + i;
    const float u = sr[tb] * xt[o];
    float x0 = u - srm1[tb] * eh[o];                 // predict_start_from_noise
    x0 = fminf(fmaxf(x0, -1.0f), 1.0f);              // clip_x_start
    const float pn = (u - x0) / srm1[tb];            // predict_noise_from_start
    g[o] = pn - eps[o];
}

template <int KH>
void launch_conv_ig(dim3 grid, hipStream_t st, const IgArgs &a)
{
    switch (a.d.in_mode) {
    case RDQ_IN_UPSAMPLE2: hipLaunchKernelGGL(HIP_KERNEL_NAME(k_conv_ig<KH, RDQ_IN_UPSAMPLE2>), grid, dim3(256), 0, st, a); break;
    case RDQ_IN_UNSHUFFLE2: hipLaunchKernelGGL(HIP_KERNEL_NAME(k_conv_ig<KH, RDQ_IN_UNSHUFFLE2>), grid, dim3(256), 0, st, a); break;
    default: hipLaunchKernelGGL(HIP_KERNEL_NAME(k_conv_ig<KH, RDQ_IN_PLAIN>), grid, dim3(256), 0, st, a); break;
    }
}


// ------------------------------------------------------------------------------- conv2d, bf16
// Mixed-precision implicit GEMM for large batches (configs[4]: hundreds of 72x72 tiles per
// iteration): bf16 operands (activations rounded to bf16 as they are staged, weights pre-packed once
// by k_pack_w_bf16), fp32 accumulation on v_mfma_f32_32x32x16_bf16 (16x the fp32 matrix rate).
// The reduction runs tap-major, k = tap * cinp + ci (cinp = cin rounded up to 32; the packed weights
// are zero-padded), so one 32-deep K stage is ONE filter tap over 32 consecutive channels: a thread
// gathers 16 channels of its pixel at a fixed stride with one bounds check per stage.
// Tile: 128 pixels (4 waves x 32: the B operand, pixel on the lane, so every accumulator register
// stores 32 consecutive pixels of one output channel) x 32*NB output channels (the A operand).
// mfma_f32_32x32x16_bf16 lane maps: A[row l&31][k 8(l>>5)+j], B[k 8(l>>5)+j][col l&31],
// D[row (r&3) + 8(r>>2) + 4(l>>5)][col l&31] (cdna_hip_programming.md §3).
constexpr int BF_BM = 128, BF_BK = 32, BF_LD = BF_BK + 8;   // LDS rows of 80 B

struct BfArgs {
    rdq_conv_desc d;
    const float *x, *x2, *bias, *res;
    const __bf16 *w;                 // [cout][taps][cinp]
    float *y, *part;
    int cinp, K, M, HW, nsteps, per_split, S;
};

__global__ __launch_bounds__(256) void k_pack_w_bf16(int cout, int cin, int taps, int cinp,
                                                     const float *__restrict__ w, __bf16 *__restrict__ wp)
{
    const int64_t n = (int64_t)cout * taps * cinp;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t o = i / ((int64_t)taps * cinp);
        const int r = (int)(i - o * taps * cinp), tap = r / cinp, ci = r - tap * cinp;
        wp[i] = ci < cin ? (__bf16)w[(o * cin + ci) * taps + tap] : (__bf16)0.0f;
    }
}

template <int MODE, int NB>
__global__ __launch_bounds__(256, 2) void k_conv_bf16(BfArgs a)
{
    constexpr int BN = 32 * NB;
    __shared__ __attribute__((aligned(16))) __bf16 Ws[2][BN][BF_LD];
    __shared__ __attribute__((aligned(16))) __bf16 As[2][BF_BM][BF_LD];
    const rdq_conv_desc &d = a.d;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int m0 = blockIdx.x * BF_BM, n0 = blockIdx.y * BN, split = blockIdx.z;
    const int s_begin = split * a.per_split, s_end = min(a.nsteps, s_begin + a.per_split);
    const int cin = d.cin1 + d.cin2, cch = a.cinp / BF_BK;
    // gather role: pixel gp, channels 16 gc .. 16 gc + 15 of the stage (gc is wave-uniform)
    const int gp = tid & (BF_BM - 1), gc = tid >> 7;
    const int gm = m0 + gp;
    const bool pv = gm < a.M;
    const int gb = pv ? gm / a.HW : 0, gpix = pv ? gm - gb * a.HW : 0;
    const int oh = gpix / d.W, ow = gpix - oh * d.W;
    // weight role: rows wn + 64 j, k octet wq (eight consecutive lanes: one octet of eight consecutive
    // rows, so each ds_write_b128 group lands on eight disjoint 16-B slots; k_conv3_bf16)
    const int wn = (tid & 7) + 8 * (tid >> 5), wq = ((tid >> 3) & 3) * 8;
    float ra[16];
    bf16x8 rw[NB / 2];
    auto load = [&](int s) {
        const int tap = s / cch, c0 = (s - tap * cch) * BF_BK + 16 * gc;
        const int ky = tap / d.kw, kx = tap - ky * d.kw;
        const int ih = oh + ky - d.pad, iw = ow + kx - d.pad;
        const bool ok = pv && (unsigned)ih < (unsigned)d.H && (unsigned)iw < (unsigned)d.W;
        if constexpr (MODE == RDQ_IN_UPSAMPLE2) {
            const int w2 = d.W >> 1;
            const size_t hw2 = (size_t)(d.H >> 1) * w2;
            const float *p = a.x + ((size_t)gb * d.cin1 + c0) * hw2 + (ok ? (ih >> 1) * w2 + (iw >> 1) : 0);
            if (c0 + 16 <= d.cin1) {                 // wave-uniform: loads without per-element tests
#pragma unroll
                for (int j = 0; j < 16; ++j) { const float v = p[j * hw2]; ra[j] = ok ? v : 0.0f; }
            } else {
#pragma unroll
                for (int j = 0; j < 16; ++j) ra[j] = (ok && c0 + j < d.cin1) ? p[j * hw2] : 0.0f;
            }
        } else if constexpr (MODE == RDQ_IN_UNSHUFFLE2) {
            const int W2 = 2 * d.W;
            const size_t hw4 = (size_t)4 * d.H * d.W;           // one plane of the full-res input
            const float *p = a.x + (size_t)gb * (d.cin1 >> 2) * hw4 + (ok ? (2 * ih) * W2 + 2 * iw : 0);
            if (c0 + 16 <= d.cin1) {
#pragma unroll
                for (int j = 0; j < 16; ++j) {       // channel c0 + j = 4c + 2 p1 + p2
                    const int ci = c0 + j;
                    const float v = p[(size_t)(ci >> 2) * hw4 + ((ci >> 1) & 1) * W2 + (ci & 1)];
                    ra[j] = ok ? v : 0.0f;
                }
            } else {
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const int ci = c0 + j;
                    ra[j] = (ok && ci < d.cin1) ? p[(size_t)(ci >> 2) * hw4 + ((ci >> 1) & 1) * W2 + (ci & 1)] : 0.0f;
                }
            }
        } else {
            const size_t hw = (size_t)d.H * d.W;
            const int off = ok ? ih * d.W + iw : 0;
            if (c0 + 16 <= d.cin1) {
                const float *p = a.x + ((size_t)gb * d.cin1 + c0) * hw + off;
#pragma unroll
                for (int j = 0; j < 16; ++j) { const float v = p[j * hw]; ra[j] = ok ? v : 0.0f; }
            } else if (c0 >= d.cin1 && c0 + 16 <= cin) {  // wave-uniform: all from the skip tensor
                const float *p = a.x2 + ((size_t)gb * d.cin2 + (c0 - d.cin1)) * hw + off;
#pragma unroll
                for (int j = 0; j < 16; ++j) { const float v = p[j * hw]; ra[j] = ok ? v : 0.0f; }
            } else {
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const int ci = c0 + j;
                    float v = 0.0f;
                    if (ok && ci < d.cin1) v = a.x[((size_t)gb * d.cin1 + ci) * hw + off];
                    else if (ok && ci < cin) v = a.x2[((size_t)gb * d.cin2 + (ci - d.cin1)) * hw + off];
                    ra[j] = v;
                }
            }
        }
#pragma unroll
        for (int j = 0; j < NB / 2; ++j) {
            const int n = n0 + wn + 64 * j;
            bf16x8 v = {};
            if (n < d.cout) v = *reinterpret_cast<const bf16x8 *>(a.w + (size_t)n * a.K + (size_t)s * BF_BK + wq);
            rw[j] = v;
        }
    };
    auto stash = [&](int buf) {
        bf16x8 v0, v1;
#pragma unroll
        for (int j = 0; j < 8; ++j) { v0[j] = (__bf16)ra[j]; v1[j] = (__bf16)ra[8 + j]; }
        *reinterpret_cast<bf16x8 *>(&As[buf][gp][16 * gc]) = v0;
        *reinterpret_cast<bf16x8 *>(&As[buf][gp][16 * gc + 8]) = v1;
#pragma unroll
        for (int j = 0; j < NB / 2; ++j) *reinterpret_cast<bf16x8 *>(&Ws[buf][wn + 64 * j][wq]) = rw[j];
    };
    f32x16 acc[NB];
#pragma unroll
    for (int c = 0; c < NB; ++c) acc[c] = f32x16{};
    if (s_begin < s_end) {
        load(s_begin);
        stash(0);
    }
    __syncthreads();
    for (int s = s_begin; s < s_end; ++s) {
        const int buf = (s - s_begin) & 1;
        if (s + 1 < s_end) load(s + 1);
#pragma unroll
        for (int ks = 0; ks < BF_BK / 16; ++ks) {
            const int kk = 16 * ks + 8 * (lane >> 5);
            const bf16x8 bv = *reinterpret_cast<const bf16x8 *>(&As[buf][wv * 32 + (lane & 31)][kk]);
#pragma unroll
            for (int c = 0; c < NB; ++c) {
                const bf16x8 av = *reinterpret_cast<const bf16x8 *>(&Ws[buf][c * 32 + (lane & 31)][kk]);
                acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc[c], 0, 0, 0);
            }
        }
        if (s + 1 < s_end) stash(buf ^ 1);
        __syncthreads();
    }
    const int m = m0 + wv * 32 + (lane & 31);
    if (m >= a.M) return;
    const int b = m / a.HW, pix = m - b * a.HW;
    const size_t slab = (size_t)a.M * d.cout;
    // residual and bias of ALL the lane's outputs are loaded before the first store (clamped
    // addresses, conditions hoisted), and every output value is formed before it: gfx9 retires
    // loads and stores in one in-order count, so a load issued after a store -- or consumed inside
    // a store's branch -- would wait for the stores already issued (a store round trip per block)
    if (a.S == 1 && (a.res || a.bias)) {
        float rv[NB][16] = {}, bv[NB][16] = {};
        if (a.bias) {
#pragma unroll
            for (int c = 0; c < NB; ++c)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    bv[c][r] = a.bias[min(n0 + c * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5), d.cout - 1)];
        }
        if (a.res) {
#pragma unroll
            for (int c = 0; c < NB; ++c)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int n = min(n0 + c * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5), d.cout - 1);
                    rv[c][r] = a.res[((size_t)b * d.cout + n) * a.HW + pix];
                }
        }
#pragma unroll
        for (int c = 0; c < NB; ++c)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[c][r] = (acc[c][r] + bv[c][r]) + rv[c][r];
    }
#pragma unroll
    for (int c = 0; c < NB; ++c)
#pragma unroll
        for (int r = 0; r < 16; ++r) asm volatile("" : "+v"(acc[c][r]));
    float *dst = a.S == 1 ? a.y : a.part + split * slab;
#pragma unroll
    for (int c = 0; c < NB; ++c)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int n = n0 + c * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            if (n < d.cout) dst[((size_t)b * d.cout + n) * a.HW + pix] = acc[c][r];
        }
}

// ------------------------------------------------------------- conv2d 3x3, bf16, halo-staged
// The per-tap kernel above re-gathers the input for each of the nine taps and waits one global
// round trip per 32-deep K stage: at the batched U-Net's sizes (configs[4]: 344 tiles) that latency,
// not the MFMA, sets its rate.  Here a workgroup owns 256 consecutive output pixels (flattened
// b, h, w) x 64 output channels and walks the reduction chunk-major: the input of a 32-channel chunk
// is gathered ONCE into LDS as the tile's halo in flattened pixel space -- rows m0 - W - 1 ..
// m0 + 256 + W, so tap (ky, kx) of output m reads halo row (m - m0) + ky W + kx -- and the nine taps
// run from it; a lane zeroes its B fragment where the tap leaves the image (the flattened neighbour
// is the wrong pixel there).  Weights stream per tap through a two-slot LDS ring, fetched two taps
// ahead; the next chunk's halo is gathered (seven 8-channel items over taps 0-4, each rounded to bf16
// and stored four taps after its loads) into the other of two LDS halo buffers while this chunk's
// MFMAs run.  4 waves x (64 pixels x 64 channels): 64
// accumulator registers, two waves per SIMD.  Halo rows are 80 B (BF_LD): the lanes of every
// ds_read_b128 group read 16 consecutive rows, conflict-free at that stride.
constexpr int C3_BM = 256, C3_BN = 64, C3_NI = 7, C3_WMAX = 72;
constexpr int C3_ROWS = C3_BM + 2 * C3_WMAX + 2;  // 402 <= 64 * C3_NI
// Zero rows C3_ZROW .. C3_ZROW + 15 of the halo buffers: a lane whose tap leaves the image reads zero
// row (its regular row & 15).  With 80-B rows a row's 16-B slot in the 64 banks is 5 row mod 16, so the
// zero row sits on the slot the lane's regular row would have used and the ds_read_b128 groups stay
// conflict-free at image borders (one shared zero row put every border lane on one slot: 2-way).
constexpr int C3_ZROW = 416;
static_assert(C3_ZROW % 16 == 0 && C3_ZROW >= C3_ROWS, "zero rows: 16-aligned, past the halo rows");

struct C3Args {
    rdq_conv_desc d;
    const float *x, *x2, *bias, *res;
    const __bf16 *x8;                // IN8: the input as bf16 octets [B][cin / 8][H W][8] (cin2 = 0)
    const __bf16 *w;                 // [cout][9][cinp]
    const float *wf;                 // k_conv3_f32: the fp32 weights in torch's own layout [cout][cin][3][3]
    float *y;
    __bf16 *yb;                      // non-null: the output rounded to bf16 and stored here instead of y
                                     // (the GroupNorm statistics are then those of the rounded values)
    double *gnp;                     // non-null: GroupNorm(G) partial statistics per (m tile, group, slot)
    int cinp, K, M, HW, R, cch, plane, G;
};

// the halo-staged convs' epilogue (k_conv3_bf16, k_conv3_f32): bias, residual, the store (fp32, or
// rounded to bf16 when a.yb is set) and the tile's GroupNorm partial statistics.  halo: the kernel's
// halo buffers (free after the last chunk's barrier; >= 32 KiB); c3g: [8-channel block][slot][s, q].
__device__ __forceinline__ void c3_epilogue(const C3Args &a, f32x16 (&acc)[2][2], const int (&pl)[2], void *halo,
                                            double (*c3g)[2][2])
{
    const rdq_conv_desc &d = a.d;
    const int tid = threadIdx.x, lane = tid & 63;
    const int m0 = blockIdx.x * C3_BM, n0 = blockIdx.y * C3_BN;
    // epilogue: the bias and residual of all 64 outputs of the lane are loaded before the first
    // store (gfx9 retires stores and loads in one in-order count: a load issued after a store would
    // wait for it), then every output is formed, then stored
    // outputs, residual and bias go through buffer resources: the lane's part of an element offset
    // (sample, its channel quad, pixel) is one VGPR per m block, the rest (the register's channel)
    // the SGPR soffset; rows past the image get an out-of-range offset (stores dropped, loads 0)
    int vo[2];
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
        const int m = m0 + pl[mb];
        const int ob = m / a.HW, opix = m - ob * a.HW;
        vo[mb] = m < a.M ? (ob * d.cout + 4 * (lane >> 5)) * a.HW + opix : -1;
    }
    auto soff = [&](int c, int r) { return (n0 + c * 32 + (r & 3) + 8 * (r >> 2)) * a.HW; };
    constexpr int OOB = (int)0x80000000u;
    float bv[2][16] = {}, rv[2][2][16] = {};
    if (a.bias) {                       // (conditions hoisted: a per-element "load or 0" would make
#pragma unroll                          //  the compiler branch and wait around every load)
        for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int r = 0; r < 16; ++r) bv[c][r] = a.bias[n0 + c * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)];
    }
    if (a.res) {
        const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(a.res), (short)0,
                                                                            0x7fffffff, 0x00020000);
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int r = 0; r < 16; ++r)
#pragma unroll
                for (int mb = 0; mb < 2; ++mb)
                    rv[mb][c][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                        rr, vo[mb] < 0 ? OOB : vo[mb] * 4, soff(c, r) * 4, 0));
    }
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                acc[c][mb][r] = (acc[c][mb][r] + bv[c][r]) + rv[mb][c][r];
                asm volatile("" : "+v"(acc[c][mb][r]));
            }
    if (a.yb) {
        const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(a.yb, (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const __bf16 h = (__bf16)acc[c][mb][r];
                    acc[c][mb][r] = (float)h;
                    __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(unsigned short, h), ry,
                                                          vo[mb] < 0 ? OOB : vo[mb] * 2, soff(c, r) * 2, 0);
                }
    } else {
        const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(a.y, (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float v = acc[c][mb][r];     // (a bit_cast of the vector element itself stored
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), ry,   //  element 0 every time)
                                                          vo[mb] < 0 ? OOB : vo[mb] * 4, soff(c, r) * 4, 0);
                }
    }
    if (!a.gnp) return;
    // GroupNorm statistics of the tile's outputs (for k_gn_apply_t with bm = C3_BM; HW >= C3_BM so a
    // tile spans at most two samples): fp64 sum and sum of squares per 8-channel block e = c*4 + (r >> 2)
    // (a lane's 4 channels r & 3; the other half-wave holds the block's other 4) and sample slot.  Each
    // thread's partials go through the halo buffer (free after the last chunk's barrier), four blocks
    // at a time, and 16 threads per (block, slot, sum) add 16 of them each in thread order, then a
    // fixed xor tree: deterministic, no long shuffle chains of fp64 per lane.
    // [16][RS] per round (34 KiB): rows RS = 272 doubles apart, so the two (block, slot, sum) rows one
    // 32-lane ds_read_b64 group reads (combo, combo + 1) fall 32 dwords apart in the 64 banks instead
    // of on the same ones (256 apart: a 2-way conflict on every read)
    constexpr int RS = 272;
    double *red = static_cast<double *>(halo);
    const int b0 = m0 / a.HW;
    int sl[2];
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
        const int m = m0 + pl[mb];
        sl[mb] = m < a.M ? m / a.HW - b0 : -1;
    }
#pragma unroll
    for (int rd = 0; rd < 2; ++rd) {
#pragma unroll
        for (int el = 0; el < 4; ++el) {
            const int e = rd * 4 + el;
            double gs[2] = {0.0, 0.0}, gq[2] = {0.0, 0.0};
#pragma unroll
            for (int mb = 0; mb < 2; ++mb) {
                double s1 = 0.0, q1 = 0.0;
#pragma unroll
                for (int r4 = 0; r4 < 4; ++r4) {
                    const double xv = acc[e >> 2][mb][(e & 3) * 4 + r4];
                    s1 += xv;
                    q1 += xv * xv;
                }
                gs[0] += sl[mb] == 0 ? s1 : 0.0;
                gq[0] += sl[mb] == 0 ? q1 : 0.0;
                gs[1] += sl[mb] == 1 ? s1 : 0.0;
                gq[1] += sl[mb] == 1 ? q1 : 0.0;
            }
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                red[((el * 2 + k) * 2 + 0) * RS + tid] = gs[k];
                red[((el * 2 + k) * 2 + 1) * RS + tid] = gq[k];
            }
        }
        __syncthreads();
        const int combo = tid >> 4, part = tid & 15;
        double v = 0.0;
#pragma unroll
        for (int j = 0; j < 16; ++j) v += red[combo * RS + part + 16 * j];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
        if (part == 0) c3g[rd * 4 + (combo >> 2)][(combo >> 1) & 1][combo & 1] = v;
        __syncthreads();
    }
    const int cpg = d.cout / a.G, gt = C3_BN / cpg, epg = cpg / 8;
    if (tid < 2 * gt) {
        const int g = tid >> 1, k = tid & 1;
        double s = 0.0, q = 0.0;
        for (int e = g * epg; e < (g + 1) * epg; ++e) {
            s += c3g[e][k][0];
            q += c3g[e][k][1];
        }
        double *o = a.gnp + (((size_t)blockIdx.x * a.G + n0 / cpg + g) * 2 + k) * 2;
        o[0] = s;
        o[1] = q;
    }
}

template <int MODE, bool IN8 = false>
__global__ __launch_bounds__(256, 2) void k_conv3_bf16(C3Args a)
{
    // row C3_ROWS of each buffer stays zero: a lane whose tap leaves the image reads it (one address
    // select per tap instead of zeroing the fragment's four registers per k step).  (The bank-matched
    // zero rows of k_conv3_f32 remove this kernel's remaining conflicts too, but the extra row
    // arithmetic spills here or, kept per tap, costs more than the conflicts: 252 -> 256 us at l72 x
    // 344 tiles, profiles/r5/pmc_conv3_bf16_zero_rows.jsonl.)
    __shared__ __attribute__((aligned(16))) __bf16 Hs[2][C3_ROWS + 1][BF_LD];     // 2 x 31.5 KiB
    __shared__ __attribute__((aligned(16))) __bf16 Ws[2][C3_BN][BF_LD];
    const rdq_conv_desc &d = a.d;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int m0 = blockIdx.x * C3_BM, n0 = blockIdx.y * C3_BN;
    const int cin = d.cin1 + d.cin2;
    // halo items: wave wv gathers the chunk's 8-channel group wv (so the source tensor and the
    // channel base are wave-uniform) for halo rows q = lane + 64 k; the source pixel is packed
    // b << 20 | pix (~0u: outside the batch or past the halo -> zeros)
    unsigned it_src[C3_NI];
#pragma unroll
    for (int k = 0; k < C3_NI; ++k) {
        const int q = lane + 64 * k, p = m0 - d.W - 1 + q;
        const bool in = q < a.R && p >= 0 && p < a.M;
        const int b = in ? p / a.HW : 0, pp = in ? p - b * a.HW : 0;
        int pix = pp;
        if constexpr (MODE == RDQ_IN_UPSAMPLE2) {
            const int ih = pp / d.W, iw = pp - ih * d.W;
            pix = (ih >> 1) * (d.W >> 1) + (iw >> 1);
        }
        it_src[k] = in ? ((unsigned)b << 20 | (unsigned)pix) : ~0u;
    }
    // one item's 8 channels of chunk cc: unconditional loads at 32-bit offsets from a wave-uniform
    // base (offset 0 where the item is empty), so the compiler never waits per load; the zeroing
    // happens when the item is rounded
    // IN8: the item's 8 channels are one 16-byte load of the packed bf16 input (already rounded)
    auto hload8 = [&](int k, int cc, bf16x8 &v) -> bool {
        const unsigned s = it_src[k];
        const bool ok = s != ~0u;
        const unsigned o = ok ? (((s >> 20) * (unsigned)(d.cin1 >> 3) + (unsigned)(cc * 4 + wv)) * (unsigned)a.plane +
                                 (s & 0xfffff)) * 8u
                              : 0u;
        v = *reinterpret_cast<const bf16x8 *>(a.x8 + o);
        return ok;
    };
    // (fp32 input) the chunk's 8-channel group of the wave through a buffer resource on its first
    // channel plane: the item's sample / pixel offset in a VGPR, the channel j's plane offset in the
    // SGPR soffset (no per-load address arithmetic); an item outside the image, or channels past
    // cin, get an offset past the resource and load zeros (no per-element select)
    const int wvu = __builtin_amdgcn_readfirstlane(wv);
    auto hsrc = [&](int cc, unsigned &cstride, bool &cok) -> __amdgpu_buffer_rsrc_t {
        const int c = cc * BF_BK + 8 * wvu;
        const bool lo = c < d.cin1;
        cok = c < cin;
        cstride = (unsigned)(lo ? d.cin1 : d.cin2) * (unsigned)a.plane * 4u;
        const float *base = !cok ? a.x : lo ? a.x + (size_t)c * a.plane : a.x2 + (size_t)(c - d.cin1) * a.plane;
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(base), (short)0, 0x7fffffff, 0x00020000);
    };
    auto hload = [&](int k, const __amdgpu_buffer_rsrc_t &rs, unsigned cstride, bool cok, float (&v)[8]) {
        const unsigned s = it_src[k];
        const int vo = (s != ~0u && cok) ? (int)((s >> 20) * cstride + (s & 0xfffff) * 4u) : (int)0x80000000u;
#pragma unroll
        for (int j = 0; j < 8; ++j)
            v[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo, j * a.plane * 4, 0));
    };
    auto hpack = [&](const float (&v)[8]) -> bf16x8 {
        bf16x8 h;
#pragma unroll
        for (int j = 0; j < 8; ++j) h[j] = (__bf16)v[j];
        return h;
    };
    auto hstore = [&](int buf, int k, const bf16x8 &h) {
        const int q = lane + 64 * k;
        if (q < a.R) *reinterpret_cast<bf16x8 *>(&Hs[buf][q][8 * wv]) = h;
    };
    // weight role: row wn (of 64), 8-channel piece wq of the tap's 32.  Eight consecutive lanes take
    // the same piece of eight consecutive rows: a ds_write_b128 group (8 contiguous lanes, banks
    // (a/4) mod 32) then starts at dwords 20 r mod 32 = {0, 20, 8, 28, 16, 4, 24, 12} + 4 piece, eight
    // disjoint 16-B slots.  (Rows tid >> 2 with pieces tid & 3 put lanes 0 and 7 of every group on the
    // same slot: a 2-way conflict on every stash, ~0.8 of the kernel's 1.1 conflict cycles per LDS
    // instruction, profiles/r4/pmc_conv3_bf16_b344_after_gather.jsonl.)
    const int wn = (tid & 7) + 8 * (tid >> 5), wq = ((tid >> 3) & 3) * 8;
    const __bf16 *wrow = a.w + (size_t)(n0 + wn) * a.K + wq;
    auto wload = [&](int cc, int t) -> bf16x8 {
        return *reinterpret_cast<const bf16x8 *>(wrow + t * a.cinp + cc * BF_BK);
    };
    auto wstash = [&](int buf, const bf16x8 &v) { *reinterpret_cast<bf16x8 *>(&Ws[buf][wn][wq]) = v; };
    // MFMA role: wave wv owns pixels wv*64 + mb*32 + (lane & 31), mb = 0, 1; bit ky*3+kx of tmask[mb]
    // says whether tap (ky, kx) stays inside the image for this lane's pixel
    int pl[2];
    unsigned tmask[2];
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
        pl[mb] = wv * 64 + mb * 32 + (lane & 31);
        const int m = m0 + pl[mb];
        const int pix = m < a.M ? m % a.HW : 0, oh = pix / d.W, ow = pix - oh * d.W;
        unsigned bits = 0;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const int ih = oh + t / 3 - 1, iw = ow + t % 3 - 1;
            bits |= ((unsigned)ih < (unsigned)d.H && (unsigned)iw < (unsigned)d.W) ? 1u << t : 0u;
        }
        tmask[mb] = m < a.M ? bits : 0u;
    }
    const int kh = 8 * (lane >> 5);
    f32x16 acc[2][2];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int mb = 0; mb < 2; ++mb) acc[c][mb] = f32x16{};

    if constexpr (IN8) {   // chunk 0's halo
        bf16x8 v[C3_NI];
        bool ok[C3_NI];
#pragma unroll
        for (int k = 0; k < C3_NI; ++k) ok[k] = hload8(k, 0, v[k]);
#pragma unroll
        for (int k = 0; k < C3_NI; ++k) hstore(0, k, ok[k] ? v[k] : bf16x8{});
    } else {
        float v[C3_NI][8];
        unsigned cs;
        bool cok;
        const __amdgpu_buffer_rsrc_t rs = hsrc(0, cs, cok);
#pragma unroll
        for (int k = 0; k < C3_NI; ++k) hload(k, rs, cs, cok, v[k]);
#pragma unroll
        for (int k = 0; k < C3_NI; ++k) hstore(0, k, hpack(v[k]));
    }
    if (tid < 2 * BF_LD / 8) reinterpret_cast<bf16x8 *>(&Hs[tid / (BF_LD / 8)][C3_ROWS][0])[tid % (BF_LD / 8)] = bf16x8{};
    // weight ring: three taps in registers; tap s is fetched at tap s - 3 into the slot tap s - 3 left
    // (stashed at the end of tap s - 4) and stashed at the end of tap s - 1: two taps of latency
    bf16x8 wr[3];
    wr[0] = wload(0, 0);
    wr[1] = wload(0, 1);
    wr[2] = wload(0, 2);
    wstash(0, wr[0]);
    __syncthreads();

    // one chunk: nine taps; PF = whether the next chunk's halo is gathered meanwhile
    auto chunk = [&](int cc, auto pf) {
        constexpr bool PF = decltype(pf)::value;
        // halo item k of the next chunk: issued at tap IT[k], rounded and stored four taps later
        // (at most six items in flight: slot k % 6)
        constexpr int IT[C3_NI] = {0, 0, 1, 1, 2, 3, 4};
        float hv[IN8 ? 1 : 6][8];
        bf16x8 hv8[IN8 ? 6 : 1];
        bool hok[6];
        const int hb = cc & 1;
        unsigned ncs = 0;
        bool ncok = false;
        __amdgpu_buffer_rsrc_t nrs;
        if constexpr (PF && !IN8) nrs = hsrc(cc + 1, ncs, ncok);
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const int s = cc * 9 + t;
            wr[t % 3] = wload(min(cc + (t + 3) / 9, a.cch - 1), (t + 3) % 9);
            if constexpr (PF) {
#pragma unroll
                for (int k = 0; k < C3_NI; ++k)
                    if (IT[k] + 4 == t) {
                        if constexpr (IN8) hstore(hb ^ 1, k, hok[k % 6] ? hv8[k % 6] : bf16x8{});
                        else hstore(hb ^ 1, k, hpack(hv[k % 6]));
                    }
#pragma unroll
                for (int k = 0; k < C3_NI; ++k)
                    if (IT[k] == t) {
                        if constexpr (IN8) hok[k % 6] = hload8(k, cc + 1, hv8[k % 6]);
                        else hload(k, nrs, ncs, ncok, hv[k % 6]);
                    }
            }
            const int toff = (t / 3) * d.W + t % 3;
            const __bf16 *wsb = &Ws[s & 1][0][0];
            int hrow[2];
#pragma unroll
            for (int mb = 0; mb < 2; ++mb) hrow[mb] = ((tmask[mb] >> t) & 1u) ? pl[mb] + toff : C3_ROWS;
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const int kk = 16 * ks + kh;
                bf16x8 bfr[2], afr[2];
#pragma unroll
                for (int mb = 0; mb < 2; ++mb)
                    bfr[mb] = *reinterpret_cast<const bf16x8 *>(&Hs[hb][hrow[mb]][kk]);
#pragma unroll
                for (int c = 0; c < 2; ++c)
                    afr[c] = *reinterpret_cast<const bf16x8 *>(wsb + (c * 32 + (lane & 31)) * BF_LD + kk);
#pragma unroll
                for (int c = 0; c < 2; ++c)
#pragma unroll
                    for (int mb = 0; mb < 2; ++mb)
                        acc[c][mb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afr[c], bfr[mb], acc[c][mb], 0, 0, 0);
            }
            wstash((s + 1) & 1, wr[(t + 1) % 3]);
            __syncthreads();
        }
    };
    for (int cc = 0; cc + 1 < a.cch; ++cc) chunk(cc, std::true_type{});
    chunk(a.cch - 1, std::false_type{});

    __shared__ double c3g[8][2][2];
    c3_epilogue(a, acc, pl, &Hs[0][0][0], c3g);
}

// ------------------------------------------------------------- conv2d 3x3, fp32, halo-staged
// k_conv3_bf16's structure on the fp32 matrix cores (v_mfma_f32_32x32x2_f32: exact fp32 products,
// the reference's precision) for the batched fp32 U-Net (configs/openfwi/red-diffeq.yaml's B = 25,
// the fp32 option of configs[4]).  A 16-channel chunk's halo is 80-B rows of 16 floats (the bf16
// kernel's row bytes, so its conflict-free ds_read_b128 pattern carries over); two lane groups read
// float4s of channels 8 q + 4 g .. + 3 and feed them to four MFMA k-steps, the weights through the
// same mapping, so every channel meets its own weight once.  Weights are read in torch's layout
// (no packing pass): a thread's four channels of a tap are four loads 9 floats apart, three taps
// ahead.  The halo items of the next chunk (2 octets x 402 rows: four per thread) are issued over
// taps 0-3 and stored four taps later.  Epilogue and GroupNorm statistics: c3_epilogue.
constexpr int C3F_BK = 16, C3F_NI = 4, C3F_LD = 20;

template <int MODE>
__global__ __launch_bounds__(256, 2) void k_conv3_f32(C3Args a)
{
    __shared__ __attribute__((aligned(16))) float Hs[2][C3_ZROW + 16][C3F_LD];   // + 16 zero rows (k_conv3_bf16)
    __shared__ __attribute__((aligned(16))) float Ws[2][C3_BN][C3F_LD];
    const rdq_conv_desc &d = a.d;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int m0 = blockIdx.x * C3_BM, n0 = blockIdx.y * C3_BN;
    const int cin = d.cin1 + d.cin2;
    // halo items: octet ho of the chunk for rows q = lane + 64 (2 k + (wv >> 1)); source pixel packed
    // b << 20 | pix as in k_conv3_bf16 (~0u: outside the batch or past the halo -> zeros)
    const int ho = wv & 1;
    unsigned it_src[C3F_NI];
#pragma unroll
    for (int k = 0; k < C3F_NI; ++k) {
        const int q = lane + 64 * (2 * k + (wv >> 1)), p = m0 - d.W - 1 + q;
        const bool in = q < a.R && p >= 0 && p < a.M;
        const int b = in ? p / a.HW : 0, pp = in ? p - b * a.HW : 0;
        int pix = pp;
        if constexpr (MODE == RDQ_IN_UPSAMPLE2) {
            const int ih = pp / d.W, iw = pp - ih * d.W;
            pix = (ih >> 1) * (d.W >> 1) + (iw >> 1);
        }
        it_src[k] = in ? ((unsigned)b << 20 | (unsigned)pix) : ~0u;
    }
    // the octet's channels through a buffer resource on its first plane, as k_conv3_bf16's gather
    const int hou = __builtin_amdgcn_readfirstlane(ho);
    auto hsrc = [&](int cc, unsigned &cstride, bool &cok) -> __amdgpu_buffer_rsrc_t {
        const int c = cc * C3F_BK + 8 * hou;
        const bool lo = c < d.cin1;
        cok = c < cin;
        cstride = (unsigned)(lo ? d.cin1 : d.cin2) * (unsigned)a.plane * 4u;
        const float *base = !cok ? a.x : lo ? a.x + (size_t)c * a.plane : a.x2 + (size_t)(c - d.cin1) * a.plane;
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(base), (short)0, 0x7fffffff, 0x00020000);
    };
    auto hload = [&](int k, const __amdgpu_buffer_rsrc_t &rs, unsigned cstride, bool cok, float (&v)[8]) {
        const unsigned s = it_src[k];
        const int vo = (s != ~0u && cok) ? (int)((s >> 20) * cstride + (s & 0xfffff) * 4u) : (int)0x80000000u;
#pragma unroll
        for (int j = 0; j < 8; ++j)
            v[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, vo, j * a.plane * 4, 0));
    };
    auto hstore = [&](int buf, int k, const float (&v)[8]) {
        const int q = lane + 64 * (2 * k + (wv >> 1));
        if (q < a.R) {
            float4 *dst = reinterpret_cast<float4 *>(&Hs[buf][q][8 * ho]);
            dst[0] = float4{v[0], v[1], v[2], v[3]};
            dst[1] = float4{v[4], v[5], v[6], v[7]};
        }
    };
    // weight role: row wn (of 64), channels wq .. wq + 3 of the chunk (cin % 8 == 0: all four inside or
    // all outside the input channels)
    // (eight consecutive lanes: one piece of eight consecutive rows, conflict-free stashes as in
    // k_conv3_bf16)
    const int wn = (tid & 7) + 8 * (tid >> 5), wq = ((tid >> 3) & 3) * 4;
    const float *wrow = a.wf + (size_t)(n0 + wn) * cin * 9;
    auto wload = [&](int cc, int t) -> float4 {
        const int c = cc * C3F_BK + wq;
        const bool ok = c < cin;
        const float *pw = wrow + (ok ? c * 9 + t : 0);
        const float4 v{pw[0], pw[9], pw[18], pw[27]};
        return ok ? v : float4{0.0f, 0.0f, 0.0f, 0.0f};
    };
    auto wstash = [&](int buf, const float4 &v) { *reinterpret_cast<float4 *>(&Ws[buf][wn][wq]) = v; };
    int pl[2];
    unsigned tmask[2];
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
        pl[mb] = wv * 64 + mb * 32 + (lane & 31);
        const int m = m0 + pl[mb];
        const int pix = m < a.M ? m % a.HW : 0, oh = pix / d.W, ow = pix - oh * d.W;
        unsigned bits = 0;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const int ih = oh + t / 3 - 1, iw = ow + t % 3 - 1;
            bits |= ((unsigned)ih < (unsigned)d.H && (unsigned)iw < (unsigned)d.W) ? 1u << t : 0u;
        }
        tmask[mb] = m < a.M ? bits : 0u;
    }
    const int kg = 4 * (lane >> 5);
    f32x16 acc[2][2];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int mb = 0; mb < 2; ++mb) acc[c][mb] = f32x16{};
    {   // chunk 0's halo
        float v[C3F_NI][8];
        unsigned cs;
        bool cok;
        const __amdgpu_buffer_rsrc_t rs = hsrc(0, cs, cok);
#pragma unroll
        for (int k = 0; k < C3F_NI; ++k) hload(k, rs, cs, cok, v[k]);
#pragma unroll
        for (int k = 0; k < C3F_NI; ++k) hstore(0, k, v[k]);
    }
    if (tid < 2 * 16 * C3F_LD / 4)
        reinterpret_cast<float4 *>(&Hs[tid / (16 * C3F_LD / 4)][C3_ZROW][0])[tid % (16 * C3F_LD / 4)] = float4{0.0f, 0.0f, 0.0f, 0.0f};
    float4 wr[3];
    wr[0] = wload(0, 0);
    wr[1] = wload(0, 1);
    wr[2] = wload(0, 2);
    wstash(0, wr[0]);
    __syncthreads();

    auto chunk = [&](int cc, auto pf) {
        constexpr bool PF = decltype(pf)::value;
        float hv[C3F_NI][8];
        const int hb = cc & 1;
        unsigned ncs = 0;
        bool ncok = false;
        __amdgpu_buffer_rsrc_t nrs;
        if constexpr (PF) nrs = hsrc(cc + 1, ncs, ncok);
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const int s = cc * 9 + t;
            wr[t % 3] = wload(min(cc + (t + 3) / 9, a.cch - 1), (t + 3) % 9);
            if constexpr (PF) {
                if (t >= 4 && t < 4 + C3F_NI) hstore(hb ^ 1, t - 4, hv[t - 4]);
                if (t < C3F_NI) hload(t, nrs, ncs, ncok, hv[t]);
            }
            const int toff = (t / 3) * d.W + t % 3;
            const float *wsb = &Ws[s & 1][0][0];
            int hrow[2];
            // bank-matched zero row (C3_ZROW): pl[mb] = 64 wv + 32 mb + (lane & 31), so the regular row's
            // residue mod 16 is the same for both mb
            const int zr = (((lane & 15) + toff) & 15) | C3_ZROW;
#pragma unroll
            for (int mb = 0; mb < 2; ++mb) hrow[mb] = ((tmask[mb] >> t) & 1u) ? pl[mb] + toff : zr;
#pragma unroll
            for (int q2 = 0; q2 < 2; ++q2) {
                const int kk = 8 * q2 + kg;
                float4 bfr[2], afr[2];
#pragma unroll
                for (int mb = 0; mb < 2; ++mb) bfr[mb] = *reinterpret_cast<const float4 *>(&Hs[hb][hrow[mb]][kk]);
#pragma unroll
                for (int c = 0; c < 2; ++c)
                    afr[c] = *reinterpret_cast<const float4 *>(wsb + (c * 32 + (lane & 31)) * C3F_LD + kk);
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int c = 0; c < 2; ++c)
#pragma unroll
                        for (int mb = 0; mb < 2; ++mb)
                            acc[c][mb] = __builtin_amdgcn_mfma_f32_32x32x2f32(afr[c][j], bfr[mb][j], acc[c][mb], 0, 0, 0);
            }
            wstash((s + 1) & 1, wr[(t + 1) % 3]);
            __syncthreads();
        }
    };
    for (int cc = 0; cc + 1 < a.cch; ++cc) chunk(cc, std::true_type{});
    chunk(a.cch - 1, std::false_type{});
    __shared__ double c3g[8][2][2];
    c3_epilogue(a, acc, pl, &Hs[0][0][0], c3g);
}

// ------------------------------------------------------ stem conv (7 x 7, one input channel)
// Unet.init_conv = Conv2d(1, 64, 7, padding=3) of the batched bf16 U-Net (an fp32 conv there: its K =
// 49 is below the bf16 path's floor).  The implicit GEMM spends its time gathering 49 taps of one
// channel per K step; here a thread owns one output pixel and all 64 channels: its 7 x 7 window from
// an LDS copy of the tile's input rows, the weights from LDS as broadcast reads (four channels per
// ds_read_b128), 3136 FMAs, 64 coalesced stores.  Workgroup: 256 consecutive pixels of one sample.
constexpr int ST_K = 7, ST_C = 64, ST_ROWS = 12;   // input rows a 256-pixel tile reads (W >= 64)
__global__ __launch_bounds__(256) void k_stem7(int H, int W, const float *__restrict__ x, const float *__restrict__ w,
                                               const float *__restrict__ bias, float *__restrict__ y)
{
    __shared__ float xs[ST_ROWS][C3_WMAX + ST_K - 1];
    __shared__ __attribute__((aligned(16))) float ws_[ST_K * ST_K][ST_C];   // [tap][channel]: broadcast reads
    const int b = blockIdx.y, HW = H * W, p0 = blockIdx.x * 256, p = p0 + (int)threadIdx.x;
    for (int i = threadIdx.x; i < ST_K * ST_K * ST_C; i += 256) {
        const int c = i / (ST_K * ST_K), t = i - c * ST_K * ST_K;
        ws_[t][c] = w[i];
    }
    const int r0 = p0 / W - ST_K / 2;                  // first input row of the window set
    const float *xb = x + (size_t)b * HW;
    for (int i = threadIdx.x; i < ST_ROWS * (W + ST_K - 1); i += 256) {
        const int rr = i / (W + ST_K - 1), cc = i - rr * (W + ST_K - 1);
        const int ih = r0 + rr, iw = cc - ST_K / 2;
        xs[rr][cc] = (ih >= 0 && ih < H && iw >= 0 && iw < W) ? xb[ih * W + iw] : 0.0f;
    }
    __syncthreads();
    if (p >= HW) return;
    const int oh = p / W, ow = p - oh * W, lr = oh - ST_K / 2 - r0;   // local row of the window top
    float acc[ST_C];
#pragma unroll
    for (int c = 0; c < ST_C; ++c) acc[c] = bias ? bias[c] : 0.0f;
#pragma unroll
    for (int ky = 0; ky < ST_K; ++ky)
#pragma unroll
        for (int kx = 0; kx < ST_K; ++kx) {
            const float v = xs[lr + ky][ow + kx];
            const f32x4 *wt = reinterpret_cast<const f32x4 *>(&ws_[ky * ST_K + kx][0]);
#pragma unroll
            for (int c4 = 0; c4 < ST_C / 4; ++c4) {
                const f32x4 w4 = wt[c4];
#pragma unroll
                for (int q = 0; q < 4; ++q) acc[4 * c4 + q] = fmaf(v, w4[q], acc[4 * c4 + q]);
            }
        }
    float *yb = y + (size_t)b * ST_C * HW + p;
#pragma unroll
    for (int c = 0; c < ST_C; ++c) yb[(size_t)c * HW] = acc[c];
}

// k_stem7 with two horizontally adjacent pixels per thread (even W): every weight read and every packed
// FMA (v_pk_fma_f32: IEEE fma per half) serves both pixels, each pixel's taps in k_stem7's order, so the
// outputs are k_stem7's bit for bit with half its LDS reads and VALU instructions per pixel.
constexpr int ST_ROWS2 = 16;                          // input rows a 512-pixel tile reads (W >= 64)
__global__ __launch_bounds__(256) void k_stem7x2(int H, int W, const float *__restrict__ x, const float *__restrict__ w,
                                                 const float *__restrict__ bias, float *__restrict__ y)
{
    typedef float f2 __attribute__((ext_vector_type(2)));
    __shared__ float xs[ST_ROWS2][C3_WMAX + ST_K];
    __shared__ __attribute__((aligned(16))) float ws_[ST_K * ST_K][ST_C];   // [tap][channel]: broadcast reads
    const int b = blockIdx.y, HW = H * W, p0 = blockIdx.x * 512, p = p0 + 2 * (int)threadIdx.x;
    for (int i = threadIdx.x; i < ST_K * ST_K * ST_C; i += 256) {
        const int c = i / (ST_K * ST_K), t = i - c * ST_K * ST_K;
        ws_[t][c] = w[i];
    }
    const int r0 = p0 / W - ST_K / 2;
    const float *xb = x + (size_t)b * HW;
    for (int i = threadIdx.x; i < ST_ROWS2 * (W + ST_K - 1); i += 256) {
        const int rr = i / (W + ST_K - 1), cc = i - rr * (W + ST_K - 1);
        const int ih = r0 + rr, iw = cc - ST_K / 2;
        xs[rr][cc] = (ih >= 0 && ih < H && iw >= 0 && iw < W) ? xb[ih * W + iw] : 0.0f;
    }
    __syncthreads();
    if (p >= HW) return;                              // HW even: p + 1 < HW too, in the same row
    const int oh = p / W, ow = p - oh * W, lr = oh - ST_K / 2 - r0;
    f2 acc[ST_C];
#pragma unroll
    for (int c = 0; c < ST_C; ++c) { const float bv = bias ? bias[c] : 0.0f; acc[c] = f2{bv, bv}; }
#pragma unroll
    for (int ky = 0; ky < ST_K; ++ky)
#pragma unroll
        for (int kx = 0; kx < ST_K; ++kx) {
            const f2 v = {xs[lr + ky][ow + kx], xs[lr + ky][ow + kx + 1]};
            const f32x4 *wt = reinterpret_cast<const f32x4 *>(&ws_[ky * ST_K + kx][0]);
#pragma unroll
            for (int c4 = 0; c4 < ST_C / 4; ++c4) {
                const f32x4 w4 = wt[c4];
#pragma unroll
                for (int q = 0; q < 4; ++q) acc[4 * c4 + q] = __builtin_elementwise_fma(v, f2{w4[q], w4[q]}, acc[4 * c4 + q]);
            }
        }
    float *yb = y + (size_t)b * ST_C * HW + p;
#pragma unroll
    for (int c = 0; c < ST_C; ++c) *reinterpret_cast<f2 *>(yb + (size_t)c * HW) = acc[c];
}

// ------------------------------------------------- linear attention, bf16, whole block fused
// LinearAttention.forward(x) + x (reference diffusion.py:182-195 and the residual at 286 / 297) for the
// batched bf16 U-Net (configs[4]: hundreds of 72 x 72 tiles).  The unfused form writes and re-reads
// qkv (384 channels, 6x the block's input) and the hidden tensor; here two launches read the input
// twice and write the output once:
//   k_lab_kv   per (sample, pixel chunk): RMSNorm(x) -> bf16 -> [k | v] = W_kv xn on
//              v_mfma_f32_32x32x16_bf16, k softmax over pixels folded into a running context
//              (flash style: per-channel running maximum, the context and the denominator rescaled
//              when it rises) -> per chunk (m, den, ctx^T) of every head
//   k_lab_out  per (sample, pixel chunk): the chunk partials and the memory tokens combined into the
//              normalised context (x scale), RMSNorm(x) -> q = W_q xn, softmax over d, hidden = ctx^T q,
//              y = W_out hidden + b, RMSNorm(y) * g * sqrt(dim) + x
// Wave h owns head h in every head-local stage.  The MFMA layouts are chosen so that no per-pixel or
// per-channel reduction crosses more than the lane pair (l, l ^ 32): k and v are formed TRANSPOSED
// (rows = pixels, columns = channels: a lane holds one channel over 16 pixels), so the softmax
// maximum over pixels is lane-local, and the context product ctx^T[e][d] = sum_n v[e][n] p[d][n]
// takes both operands straight from those registers (the reduction index n enumerated in the same
// register order for both); q is formed with pixels as columns (a lane holds 16 of one pixel's 32 d),
// so the softmax over d is lane-local plus one swap, and hidden = ctx^T q takes q from registers.
// Operands are bf16 (activations rounded as staged, as the bf16 convs do, and the softmax weights
// and context), every accumulation fp32.
constexpr int LB_PX = 64, LB_DH = 32, LB_HEADS = 4, LB_HID = LB_HEADS * LB_DH;
constexpr int LB_PART = LB_HEADS * (2 * LB_DH + LB_DH * LB_DH);   // floats per (sample, chunk)

struct LabArgs {
    const float *x, *g_in, *mem, *b_out, *g_out;
    const __bf16 *wqkv;              // [3 * 128][D]  (q, k, v rows)
    const __bf16 *wout;              // [D][128]
    const float *wqkv32, *wout32;    // the fp32 form (F): the module's own weights, same layouts
    float *part, *y;
    int n, nch, nsub, nmem;
    float scale;
};

// D layout of v_mfma_f32_32x32x16_bf16: register r of lane l holds row (r & 3) + 8 (r >> 2) + 4 (l >> 5)
__device__ __forceinline__ int lb_row(int r, int g) { return (r & 3) + 8 * (r >> 2) + 4 * g; }

// RMSNorm(x) of pixels [p0, p0 + 64) of sample b, rounded to bf16, into Xs[px][c], in two halves so
// the next tile's loads are in flight during this tile's MFMAs: lb_load (thread: pixel lane, channel
// octets wave + 4 j; pixels past n read pixel n - 1, their results are masked) and lb_store (the
// norm over the four waves' partial sums, then the scaled bf16 octets).  lb_store's barrier also
// orders its Xs writes after every wave's reads of the previous tile.
template <int D>
__device__ __forceinline__ void lb_load(const LabArgs &a, int b, int p0, float (&v)[D / 32][8])
{
    // buffer loads: one lane offset for every channel, the channel's plane offset in an SGPR
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int voff = min(p0 + lane, a.n - 1) * 4;
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(a.x + (size_t)b * D * a.n), (short)0, D * a.n * 4, 0x00020000);
#pragma unroll
    for (int j = 0; j < D / 32; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i)
            v[j][i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                    rx, voff, (8 * (w + 4 * j) + i) * a.n * 4, 0));
}

// staged operand rows: bf16 [px][D + 8] (16-byte fragment reads), or fp32 [px][D + 1] (F: one float
// per lane and k-step, odd pitch: conflict-free)
template <int D, bool F> struct LbX {
    using T = typename std::conditional<F, float, __bf16>::type;
    static constexpr int P = F ? D + 1 : D + 8;
};
template <int D, bool F>
__device__ __forceinline__ void lb_store(const LabArgs &a, const float (&v)[D / 32][8],
                                         typename LbX<D, F>::T (*Xs)[LbX<D, F>::P], float (*red)[LB_PX])
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float ss = 0.0f;
#pragma unroll
    for (int j = 0; j < D / 32; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) ss = fmaf(v[j][i], v[j][i], ss);
    red[w][lane] = ss;
    __syncthreads();
    const float tot = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
    const float k = sqrtf((float)D) / fmaxf(sqrtf(tot), 1e-12f);
#pragma unroll
    for (int j = 0; j < D / 32; ++j) {
        const int c0 = 8 * (w + 4 * j);
        if constexpr (F) {
#pragma unroll
            for (int i = 0; i < 8; ++i) Xs[lane][c0 + i] = v[j][i] * k * a.g_in[c0 + i];
        } else {
            bf16x8 o;
#pragma unroll
            for (int i = 0; i < 8; ++i) o[i] = (__bf16)(v[j][i] * k * a.g_in[c0 + i]);
            *reinterpret_cast<bf16x8 *>(&Xs[lane][c0]) = o;
        }
    }
}

// Occupancy sets the rate of these streaming kernels (each workgroup has one tile's loads in flight
// during the previous tile's MFMAs): register budgets of 3 (dim 64) / 2 (dim 128) workgroups per CU.
template <int D, bool F = false> struct LbOcc {      // (F: fp32 staging, LDS-bound)
    static constexpr int N = F ? (D == 64 ? 2 : 1) : (D == 64 ? 3 : 2);
};

// F: the fp32 form (the reference's arithmetic, small batches): the same structure on
// v_mfma_f32_32x32x2_f32 (k index of lane group g = g: one float per lane and k-step), fp32 staging
// softmax exponentials of the LinearAttention kernels: the bf16 form rounds its operands to bf16
// anyway, so it takes the hardware exp2 (v_exp_f32 after a scale by log2 e) instead of expf's
// range-reduced evaluation; the fp32 form keeps expf (the reference's precision)
template <bool F> __device__ __forceinline__ float lab_exp(float x) { return F ? expf(x) : __expf(x); }

template <int D, bool F = false>
__global__ __launch_bounds__(256, (LbOcc<D, F>::N)) void k_lab_kv(LabArgs a)
{
    constexpr int KS = D / 16;                       // k-steps over the input channels
    constexpr bool WREG = D <= 64 && !F;             // W_kv fragments held in registers (else L1 / L2)
    __shared__ __attribute__((aligned(16))) typename LbX<D, F>::T Xs[LB_PX][LbX<D, F>::P];
    __shared__ float red[4][LB_PX];
    const int ch = blockIdx.x, b = blockIdx.y;
    const int lane = threadIdx.x & 63, h = threadIdx.x >> 6, g = lane >> 5, cl = lane & 31;
    // B fragments: column = channel cl of head h (k rows 128 + 32 h, v rows 256 + 32 h), k = c
    const __bf16 *wk = a.wqkv + (size_t)(LB_HID + h * LB_DH + cl) * D + 8 * g;
    const __bf16 *wv = a.wqkv + (size_t)(2 * LB_HID + h * LB_DH + cl) * D + 8 * g;
    const float *wk32 = a.wqkv32 + (size_t)(LB_HID + h * LB_DH + cl) * D + g;
    const float *wv32 = a.wqkv32 + (size_t)(2 * LB_HID + h * LB_DH + cl) * D + g;
    bf16x8 fk[WREG ? KS : 1], fv[WREG ? KS : 1];
    if constexpr (WREG) {
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            fk[s] = *reinterpret_cast<const bf16x8 *>(wk + 16 * s);
            fv[s] = *reinterpret_cast<const bf16x8 *>(wv + 16 * s);
        }
    }
    f32x16 ctx = {};
    float mrun = -INFINITY, den = 0.0f;
    const int sub0 = ch * a.nsub, sub1 = min(sub0 + a.nsub, (a.n + LB_PX - 1) / LB_PX);
    float xv[D / 32][8];
    if (sub0 < sub1) lb_load<D>(a, b, sub0 * LB_PX, xv);
    for (int sb = sub0; sb < sub1; ++sb) {
        const int p0 = sb * LB_PX;
        lb_store<D, F>(a, xv, Xs, red);
        __syncthreads();
        if (sb + 1 < sub1) lb_load<D>(a, b, p0 + LB_PX, xv);
        // one 32-pixel block at a time: k^T and v^T (rows = pixels, column = channel cl), the online
        // softmax over the pixels of channel d = cl (this lane and lane ^ 32), the context update
#pragma unroll 1
        for (int pb = 0; pb < 2; ++pb) {
            f32x16 kt = {}, vt = {};
            if constexpr (F) {
#pragma unroll 8
                for (int s = 0; s < D / 2; ++s) {
                    const float av = Xs[pb * 32 + cl][2 * s + g];
                    kt = __builtin_amdgcn_mfma_f32_32x32x2f32(av, wk32[2 * s], kt, 0, 0, 0);
                    vt = __builtin_amdgcn_mfma_f32_32x32x2f32(av, wv32[2 * s], vt, 0, 0, 0);
                }
            } else {
#pragma unroll
                for (int s = 0; s < KS; ++s) {
                    const bf16x8 bk = WREG ? fk[s] : *reinterpret_cast<const bf16x8 *>(wk + 16 * s);
                    const bf16x8 bv = WREG ? fv[s] : *reinterpret_cast<const bf16x8 *>(wv + 16 * s);
                    const bf16x8 av = *reinterpret_cast<const bf16x8 *>(&Xs[pb * 32 + cl][16 * s + 8 * g]);
                    kt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bk, kt, 0, 0, 0);
                    vt = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, vt, 0, 0, 0);
                }
            }
            float tmax = -INFINITY;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const bool ok = p0 + pb * 32 + lb_row(r, g) < a.n;
                kt[r] = ok ? kt[r] : -INFINITY;
                tmax = fmaxf(tmax, kt[r]);
            }
            tmax = fmaxf(tmax, __shfl_xor(tmax, 32));
            const float mnew = fmaxf(mrun, tmax);
            const float f = mrun == -INFINITY ? 0.0f : lab_exp<F>(mrun - mnew);
            mrun = mnew;
            float ps = 0.0f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float e = kt[r] == -INFINITY ? 0.0f : lab_exp<F>(kt[r] - mnew);
                kt[r] = e;
                ps += e;
            }
            den = den * f + ps;
#pragma unroll
            for (int r = 0; r < 16; ++r) ctx[r] *= f;
            // ctx^T[e][d] += sum_n v[e][n] p[d][n]: k index j of lane group g <-> pixel lb_row(8 s + j, g)
            // (F: k index g of step r <-> pixel lb_row(r, g))
            if constexpr (F) {
#pragma unroll
                for (int r = 0; r < 16; ++r) ctx = __builtin_amdgcn_mfma_f32_32x32x2f32(vt[r], kt[r], ctx, 0, 0, 0);
            } else {
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    bf16x8 av, bp;
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        av[j] = (__bf16)vt[8 * s + j];
                        bp[j] = (__bf16)kt[8 * s + j];
                    }
                    ctx = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bp, ctx, 0, 0, 0);
                }
            }
        }
    }
    den += __shfl_xor(den, 32);
    float *o = a.part + ((size_t)b * a.nch + ch) * LB_PART + h * (2 * LB_DH + LB_DH * LB_DH);
    if (g == 0) {
        o[cl] = mrun;
        o[LB_DH + cl] = den;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) o[2 * LB_DH + lb_row(r, g) * LB_DH + cl] = ctx[r];
}

template <int D, bool F = false>
__global__ __launch_bounds__(256, (LbOcc<D, F>::N)) void k_lab_out(LabArgs a)
{
    constexpr int KS = D / 16, NOB = D / 64;         // o blocks per wave (two waves per pixel block)
    constexpr bool WREG = D <= 64 && !F, WOREG = false;   // W_q / W_out fragments in registers (else L1 / L2)
    __shared__ __attribute__((aligned(16))) typename LbX<D, F>::T Xs[LB_PX][LbX<D, F>::P];
    __shared__ __attribute__((aligned(16))) typename LbX<LB_HID, F>::T Hs[LB_PX][LbX<LB_HID, F>::P];
    __shared__ float red[4][LB_PX];
    __shared__ float red2[4][32];
    __shared__ float Cs[LB_HEADS][LB_DH][LB_DH + 1];
    const int ch = blockIdx.x, b = blockIdx.y;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = w, g = lane >> 5, cl = lane & 31;
    // ---- the normalised context of head h (x scale): chunks combined in order, then the memory tokens
    {
        const int d = cl;
        const float *mk = a.mem + ((size_t)(0 * LB_HEADS + h) * LB_DH + d) * a.nmem;
        float M = -INFINITY;
        for (int j = 0; j < a.nmem; ++j) M = fmaxf(M, mk[j]);
        const float *pb0 = a.part + (size_t)b * a.nch * LB_PART + h * (2 * LB_DH + LB_DH * LB_DH);
        for (int c = 0; c < a.nch; ++c) M = fmaxf(M, pb0[(size_t)c * LB_PART + d]);
        float den = 0.0f, acc[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
        for (int c = 0; c < a.nch; ++c) {
            const float *pc = pb0 + (size_t)c * LB_PART;
            const float mc = pc[d];
            const float f = mc == -INFINITY ? 0.0f : lab_exp<F>(mc - M);
            den += f * pc[LB_DH + d];
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] += f * pc[2 * LB_DH + lb_row(r, g) * LB_DH + d];
        }
        const float *mv = a.mem + (size_t)(1 * LB_HEADS + h) * LB_DH * a.nmem;
        for (int j = 0; j < a.nmem; ++j) {
            const float e = lab_exp<F>(mk[j] - M);
            den += e;
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[r] += e * mv[(size_t)lb_row(r, g) * a.nmem + j];
        }
        // lanes d and d + 32 both formed den (same terms): acc rows e split between them
        const float k = a.scale / den;
#pragma unroll
        for (int r = 0; r < 16; ++r) Cs[h][d][lb_row(r, g)] = acc[r] * k;
    }
    __syncthreads();
    // A fragments of hidden = ctx^T q: row e = cl, k index j of group g <-> d = lb_row(8 s + j, g)
    bf16x8 fc[F ? 1 : 2];
    float fcf[F ? 16 : 1];                           // F: step r's k index g <-> d = lb_row(r, g)
    if constexpr (F) {
#pragma unroll
        for (int r = 0; r < 16; ++r) fcf[r] = Cs[h][lb_row(r, g)][cl];
    } else {
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int j = 0; j < 8; ++j) fc[s][j] = (__bf16)Cs[h][lb_row(8 * s + j, g)][cl];
    }
    // q rows of head h (A operand, row d = cl) and the wave's W_out rows (A operand, row o)
    const __bf16 *wq = a.wqkv + (size_t)(h * LB_DH + cl) * D + 8 * g;
    const float *wq32 = a.wqkv32 + (size_t)(h * LB_DH + cl) * D + g;
    bf16x8 fq[WREG ? KS : 1];
    if constexpr (WREG) {
#pragma unroll
        for (int s = 0; s < KS; ++s) fq[s] = *reinterpret_cast<const bf16x8 *>(wq + 16 * s);
    }
    const int pbw = __builtin_amdgcn_readfirstlane(w & 1), obw = __builtin_amdgcn_readfirstlane(w >> 1);   // y tiles:
                                                     // pixel block pbw, o blocks obw + 2 j
    const __bf16 *wo = a.wout + (size_t)(obw * 32 + cl) * LB_HID + 8 * g;
    const float *wo32 = a.wout32 + (size_t)(obw * 32 + cl) * LB_HID + g;
    bf16x8 fo[WOREG ? NOB : 1][8];
    if constexpr (WOREG) {
#pragma unroll
        for (int j = 0; j < NOB; ++j)
#pragma unroll
            for (int s = 0; s < 8; ++s) fo[j][s] = *reinterpret_cast<const bf16x8 *>(wo + (size_t)j * 64 * LB_HID + 16 * s);
    }
    const float gs = sqrtf((float)D);
    const int sub0 = ch * a.nsub, sub1 = min(sub0 + a.nsub, (a.n + LB_PX - 1) / LB_PX);
    float xv[D / 32][8];
    if (sub0 < sub1) lb_load<D>(a, b, sub0 * LB_PX, xv);
    for (int sb = sub0; sb < sub1; ++sb) {
        const int p0 = sb * LB_PX;
        lb_store<D, F>(a, xv, Xs, red);              // (its barrier: Hs / red2 of the previous tile consumed)
        __syncthreads();
        if (sb + 1 < sub1) lb_load<D>(a, b, p0 + LB_PX, xv);
        // q[d][px] of head h, softmax over d (this lane's 16 d and lane ^ 32's), then hidden
#pragma unroll
        for (int pb = 0; pb < 2; ++pb) {
            f32x16 q = {};
            if constexpr (F) {
#pragma unroll 8
                for (int s = 0; s < D / 2; ++s)
                    q = __builtin_amdgcn_mfma_f32_32x32x2f32(wq32[2 * s], Xs[pb * 32 + cl][2 * s + g], q, 0, 0, 0);
            } else {
#pragma unroll
                for (int s = 0; s < KS; ++s) {
                    const bf16x8 aw = WREG ? fq[s] : *reinterpret_cast<const bf16x8 *>(wq + 16 * s);
                    const bf16x8 bx = *reinterpret_cast<const bf16x8 *>(&Xs[pb * 32 + cl][16 * s + 8 * g]);
                    q = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aw, bx, q, 0, 0, 0);
                }
            }
            float mx = -INFINITY;
#pragma unroll
            for (int r = 0; r < 16; ++r) mx = fmaxf(mx, q[r]);
            mx = fmaxf(mx, __shfl_xor(mx, 32));
            float sm = 0.0f;
#pragma unroll
            for (int r = 0; r < 16; ++r) { q[r] = lab_exp<F>(q[r] - mx); sm += q[r]; }
            sm += __shfl_xor(sm, 32);
            const float inv = 1.0f / sm;
            f32x16 hid = {};
            if constexpr (F) {
#pragma unroll
                for (int r = 0; r < 16; ++r) hid = __builtin_amdgcn_mfma_f32_32x32x2f32(fcf[r], q[r] * inv, hid, 0, 0, 0);
#pragma unroll
                for (int r = 0; r < 16; ++r) Hs[pb * 32 + cl][h * LB_DH + lb_row(r, g)] = hid[r];
            } else {
#pragma unroll
                for (int s = 0; s < 2; ++s) {
                    bf16x8 bq;
#pragma unroll
                    for (int j = 0; j < 8; ++j) bq[j] = (__bf16)(q[8 * s + j] * inv);
                    hid = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fc[s], bq, hid, 0, 0, 0);
                }
                // hidden[e][px] -> Hs[px][32 h + e]: rows 4 q4 .. 4 q4 + 3 are four consecutive e
#pragma unroll
                for (int q4 = 0; q4 < 4; ++q4) {
                    __attribute__((ext_vector_type(4))) __bf16 o4;
#pragma unroll
                    for (int i = 0; i < 4; ++i) o4[i] = (__bf16)hid[4 * q4 + i];
                    *reinterpret_cast<decltype(o4) *>(&Hs[pb * 32 + cl][h * LB_DH + lb_row(4 * q4, g)]) = o4;
                }
            }
        }
        __syncthreads();
        // y[o][px] = W_out hidden + b for pixel block pbw, o blocks obw + 2 j; the residual in flight
        const int px = p0 + pbw * 32 + cl;
        // residual loads / output stores through buffer resources of sample b: lane offset (pixel, row
        // group 4 g), the row's plane in an SGPR; pixels past n store to an offset past the buffer
        const int vo = (min(px, a.n - 1) + 4 * g * a.n) * 4;
        const int vs = px < a.n ? (px + 4 * g * a.n) * 4 : (int)0x80000000u;
        const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float *>(a.x + (size_t)b * D * a.n), (short)0, D * a.n * 4, 0x00020000);
        const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(a.y + (size_t)b * D * a.n, (short)0,
                                                                            D * a.n * 4, 0x00020000);
        float rv[NOB][16];
#pragma unroll
        for (int j = 0; j < NOB; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r)
                rv[j][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                    rx, vo, ((obw + 2 * j) * 32 + (r & 3) + 8 * (r >> 2)) * a.n * 4, 0));
        f32x16 y[NOB];
        float ss = 0.0f;
#pragma unroll
        for (int j = 0; j < NOB; ++j) {
            y[j] = f32x16{};
            if constexpr (F) {
#pragma unroll 8
                for (int s = 0; s < LB_HID / 2; ++s)
                    y[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(wo32[(size_t)j * 64 * LB_HID + 2 * s],
                                                                Hs[pbw * 32 + cl][2 * s + g], y[j], 0, 0, 0);
            } else {
#pragma unroll
                for (int s = 0; s < 8; ++s) {
                    const bf16x8 aw = WOREG ? fo[j][s]
                                            : *reinterpret_cast<const bf16x8 *>(wo + (size_t)j * 64 * LB_HID + 16 * s);
                    const bf16x8 bh = *reinterpret_cast<const bf16x8 *>(&Hs[pbw * 32 + cl][16 * s + 8 * g]);
                    y[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aw, bh, y[j], 0, 0, 0);
                }
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float t = y[j][r] + (a.b_out ? a.b_out[(obw + 2 * j) * 32 + lb_row(r, g)] : 0.0f);
                y[j][r] = t;
                ss = fmaf(t, t, ss);
            }
        }
        ss += __shfl_xor(ss, 32);
        if (g == 0) red2[w][cl] = ss;
        __syncthreads();
        const float tot = red2[pbw][cl] + red2[pbw + 2][cl];
        const float k = gs / fmaxf(sqrtf(tot), 1e-12f);
#pragma unroll
        for (int j = 0; j < NOB; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int o = (obw + 2 * j) * 32 + lb_row(r, g);
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, y[j][r] * k * a.g_out[o] + rv[j][r]),
                                                      ry, vs, ((obw + 2 * j) * 32 + (r & 3) + 8 * (r >> 2)) * a.n * 4, 0);
            }
    }
}

// the halo-staged kernel takes 3x3 / pad 1 convs (plain, with a concatenated skip, or on a nearest-
// upsampled input) with at least C3_MIN_TILES tiles; everything else stays on the per-tap kernel. The
// halo kernel wins even on a part-filled chip (bf16 U-Net forward, B = 25: 4.15 -> 3.13 ms, B = 100:
// 8.0 -> 6.2 ms, B = 344: 18.5 -> 18.1 ms going from 512 to 64); below ~64 tiles it loses at B <= 8
// Process-wide kernel options (rdq_unet_set_option).  Atomics, so a concurrent set is never torn; every
// change bumps g_opt_gen (rdq_unet_options_generation), which the Python U-Net folds into its captured-
// graph cache key, so graphs captured under the old choice are recaptured instead of replayed.
static std::atomic<int> C3_BF16_RAW{1};      // RDQ_UNET_OPT_BF16_RAW
static std::atomic<int> C3_MIN_TILES{64};    // RDQ_UNET_OPT_CONV3_MIN_TILES; tools/conv3_threshold_ab.py
static std::atomic<int> C3F_MIN_TILES{192};  // k_conv3_f32; RDQ_UNET_OPT_CONV3F_MIN_TILES, 0 = never
static std::atomic<int> g_opt_gen{0};
static int64_t conv3_tiles(const rdq_conv_desc *d)
{
    if (d->kh != 3 || d->kw != 3 || d->pad != 1) return 0;
    if (d->in_mode != RDQ_IN_PLAIN && d->in_mode != RDQ_IN_UPSAMPLE2) return false;
    if (d->cin1 % 8 || d->cin2 % 8 || d->cout % C3_BN || d->W > C3_WMAX || d->B >= 4096) return false;
    const int64_t HW = (int64_t)d->H * d->W, M = d->B * HW;
    if (HW >= (1 << 20) || M >= (int64_t)1 << 30) return false;
    // the halo gather addresses each input tensor with 31-bit byte offsets (buffer loads)
    const int64_t plane = d->in_mode == RDQ_IN_UPSAMPLE2 ? HW / 4 : HW;
    if ((int64_t)d->B * std::max(d->cin1, d->cin2) * plane * 4 >= (int64_t)1 << 31) return false;
    if (M * d->cout * 4 >= (int64_t)1 << 31) return false;     // output / residual: the same, epilogue
    return (M + C3_BM - 1) / C3_BM * (d->cout / C3_BN);
}
bool conv3_ok(const rdq_conv_desc *d) { return conv3_tiles(d) >= C3_MIN_TILES; }
bool conv3f_ok(const rdq_conv_desc *d) { return C3F_MIN_TILES > 0 && conv3_tiles(d) >= C3F_MIN_TILES; }

// k_conv3_f32 on a conv3f_ok descriptor (raw fp32 weights); gnp: GroupNorm partials (bm = C3_BM) or null
void launch_conv3_f32(const rdq_conv_desc *d, const float *x, const float *x2, const float *w, const float *bias,
                      const float *res, float *y, double *gnp, int G, hipStream_t st)
{
    C3Args c{};
    c.d = *d; c.x = x; c.x2 = x2; c.wf = w; c.bias = bias; c.res = res; c.y = y; c.gnp = gnp; c.G = G;
    c.cinp = (d->cin1 + d->cin2 + C3F_BK - 1) / C3F_BK * C3F_BK;
    c.K = 9 * c.cinp;
    c.HW = d->H * d->W;
    c.M = d->B * c.HW;
    c.R = C3_BM + 2 * d->W + 2;
    c.cch = c.cinp / C3F_BK;
    c.plane = d->in_mode == RDQ_IN_UPSAMPLE2 ? c.HW / 4 : c.HW;
    const dim3 grid((c.M + C3_BM - 1) / C3_BM, d->cout / C3_BN);
    if (d->in_mode == RDQ_IN_UPSAMPLE2)
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_conv3_f32<RDQ_IN_UPSAMPLE2>), grid, dim3(256), 0, st, c);
    else
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_conv3_f32<RDQ_IN_PLAIN>), grid, dim3(256), 0, st, c);
}

int bf_cinp(const rdq_conv_desc *d) { return (d->cin1 + d->cin2 + BF_BK - 1) / BF_BK * BF_BK; }

// split count as ig_splits: about two workgroups per CU over the tile grid, >= 4 K stages each
int bf_splits(const rdq_conv_desc *d, int BN, int nsteps, size_t ws_bytes, int *per_split)
{
    const int M = d->B * d->H * d->W;
    const int tiles = ((M + BF_BM - 1) / BF_BM) * ((d->cout + BN - 1) / BN);
    int S = std::max(1, std::min((512 + tiles - 1) / tiles, nsteps / 4));
    const size_t slab = (size_t)M * d->cout * sizeof(float);
    if (S > 1 && ws_bytes < 2 * slab) S = 1;
    if (S > 1) S = std::min<int64_t>(S, (int64_t)(ws_bytes / slab));
    const int per = (nsteps + S - 1) / S;
    *per_split = per;
    return (nsteps + per - 1) / per;
}

template <int NB>
void launch_conv_bf16(dim3 grid, hipStream_t st, const BfArgs &a)
{
    switch (a.d.in_mode) {
    case RDQ_IN_UPSAMPLE2: hipLaunchKernelGGL(HIP_KERNEL_NAME(k_conv_bf16<RDQ_IN_UPSAMPLE2, NB>), grid, dim3(256), 0, st, a); break;
    case RDQ_IN_UNSHUFFLE2: hipLaunchKernelGGL(HIP_KERNEL_NAME(k_conv_bf16<RDQ_IN_UNSHUFFLE2, NB>), grid, dim3(256), 0, st, a); break;
    default: hipLaunchKernelGGL(HIP_KERNEL_NAME(k_conv_bf16<RDQ_IN_PLAIN, NB>), grid, dim3(256), 0, st, a); break;
    }
}

// k_conv_cc for a cc_ok descriptor: 3x3 (plain / nearest x2) or 1x1 (plain / 2x2 unshuffle)
void launch_cc(const CcArgs &c, dim3 grid, hipStream_t st)
{
    const rdq_conv_desc *d = &c.d;
#define RDQ_LCC(T, M) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_conv_cc<T, M>), grid, dim3(256), 0, st, c)
    if (d->kh == 3) {
        if (d->in_mode == RDQ_IN_UPSAMPLE2) RDQ_LCC(9, RDQ_IN_UPSAMPLE2);
        else RDQ_LCC(9, RDQ_IN_PLAIN);
    } else {
        if (d->in_mode == RDQ_IN_UNSHUFFLE2) RDQ_LCC(1, RDQ_IN_UNSHUFFLE2);
        else RDQ_LCC(1, RDQ_IN_PLAIN);
    }
#undef RDQ_LCC
}

bool conv_desc_ok(const rdq_conv_desc *d)
{
    if (!d || d->B < 1 || d->cin1 < 1 || d->cout < 1 || d->kh < 1 || d->kw < 1 || d->H < 1 || d->W < 1 || d->pad < 0)
        return false;
    if (d->in_mode == RDQ_IN_UNSHUFFLE2 && (d->cin1 % 4 != 0 || d->cin2 != 0)) return false;
    if (d->in_mode == RDQ_IN_UPSAMPLE2 && ((d->H | d->W) & 1 || d->cin2 != 0)) return false;
    return true;
}
}  // namespace

// the small-image form is its own instantiation (the per-channel form's code is unchanged by it)
// (gn4: gn_grid chose 4096-element chunks: the k_gn_apply_t<false, 4> instantiation)
#define LAUNCH_GN_T(GRID, ST, ...)                                                                     \
    do {                                                                                               \
        if (nch < 0) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_gn_apply_t<true>), GRID, dim3(256), 0, ST, __VA_ARGS__); \
        else if (gn4) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_gn_apply_t<false, 4>), GRID, dim3(256), 0, ST, __VA_ARGS__); \
        else hipLaunchKernelGGL(HIP_KERNEL_NAME(k_gn_apply_t<false>), GRID, dim3(256), 0, ST, __VA_ARGS__);      \
    } while (0)
#define LAUNCH_GN_TB(GRID, ST, ...)                                                                    \
    do {                                                                                               \
        if (nch < 0) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_gn_apply_t<true, 1, __bf16>), GRID, dim3(256), 0, ST, __VA_ARGS__); \
        else if (gn4) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_gn_apply_t<false, 4, __bf16>), GRID, dim3(256), 0, ST, __VA_ARGS__); \
        else hipLaunchKernelGGL(HIP_KERNEL_NAME(k_gn_apply_t<false, 1, __bf16>), GRID, dim3(256), 0, ST, __VA_ARGS__); \
    } while (0)
#define LAUNCH_GN(GRID, ST, ...)                                                                       \
    do {                                                                                               \
        if (nch < 0) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_gn_apply<true>), GRID, dim3(256), 0, ST, __VA_ARGS__);   \
        else hipLaunchKernelGGL(HIP_KERNEL_NAME(k_gn_apply<false>), GRID, dim3(256), 0, ST, __VA_ARGS__);        \
    } while (0)

// GroupNorm pass grid: one workgroup per (channel, 1024-element chunk) of a group, or for images of
// <= 512 pixels in grids of more than 8192 workgroups -nch = 1024 / HW whole channels per workgroup
// (9 x 9 at B = 344 had 176 K workgroups of 81 elements each: 138 -> 10 us per pass; at B = 1 the
// per-channel form is faster); returns the x extent, *nch the kernels' chunk argument.  With gn4
// (callers of k_gn_apply_t only) batched sizes of >= 16 M elements take 4096-element chunks
static int gn_grid(int B, int C, int G, int HW, int *nch, bool *gn4 = nullptr)
{
    const int cpg = C / G;
    if (gn4) *gn4 = false;
    if (HW <= 512 && (int64_t)C * B > 8192) {
        const int cpb = 1024 / HW;
        *nch = -cpb;
        return (cpg + cpb - 1) / cpb;
    }
    const int chunk = gn4 && (int64_t)B * C * HW >= (1 << 24) ? 4096 : 1024;
    if (gn4) *gn4 = chunk == 4096;
    *nch = (HW + chunk - 1) / chunk;
    return cpg * *nch;
}

extern "C" {

size_t rdq_conv2d_tickets(const rdq_conv_desc *d)
{
    if (!d || d->B < 1 || d->H < 1 || d->W < 1 || d->cout < 1) return 0;
    const int64_t M = (int64_t)d->B * d->H * d->W;
    return (size_t)(((M + CC_BM - 1) / CC_BM) * ((d->cout + CC_BN - 1) / CC_BN));
}

size_t rdq_conv2d_ws_bytes(const rdq_conv_desc *d)
{
    if (!d || d->B < 1 || d->H < 1 || d->W < 1 || d->cout < 1 || d->kh < 1 || d->kw < 1 || d->cin1 < 1) return 0;
    int per = 0;
    if (cc_ok(d)) {
        const int S = cc_splits(d, (size_t)-1 / 2, &per);
        return S > 1 ? (size_t)S * rdq_conv2d_tickets(d) * CC_BM * CC_BN * sizeof(float) : 0;
    }
    const int S = ig_splits(d, (size_t)-1 / 2, &per);
    return S > 1 ? (size_t)S * d->B * d->H * d->W * d->cout * sizeof(float) : 0;
}


int rdq_conv2d(const rdq_conv_desc *d, const float *x, const float *x2, const float *w, const float *bias,
               const float *residual, float *y, void *ws, size_t ws_bytes, uint32_t *tickets, hipStream_t st)
{
    if (!d || !x || !w || !y || d->B < 1 || d->cin1 < 1 || d->cout < 1 || d->kh < 1 || d->kw < 1 || d->H < 1 ||
        d->W < 1 || d->pad < 0 || (d->cin2 > 0 && !x2 && d->in_mode == RDQ_IN_PLAIN))
        return RDQ_E_INVALID;
    if (d->in_mode == RDQ_IN_UNSHUFFLE2 && (d->cin1 % 4 != 0 || d->cin2 != 0)) return RDQ_E_INVALID;
    if (d->in_mode == RDQ_IN_UPSAMPLE2 && ((d->H | d->W) & 1 || d->cin2 != 0)) return RDQ_E_INVALID;
    if (conv3f_ok(d)) {
        launch_conv3_f32(d, x, x2, w, bias, residual, y, nullptr, 0, st);
        RDQ_CHECK(hipGetLastError());
        return 0;
    }
    if (cc_ok(d)) {
        CcArgs c{};
        c.d = *d; c.x = x; c.x2 = x2; c.w = w; c.bias = bias; c.res = residual; c.y = y;
        c.part = static_cast<float *>(ws);
        c.tickets = tickets;
        c.K = (d->cin1 + d->cin2) * d->kh * d->kw;
        c.HW = d->H * d->W;
        c.M = d->B * c.HW;
        cc_extents(c, d);
        c.nstages = (d->cin1 + d->cin2) / (d->kh == 3 ? CcCfg<9>::CPS : CcCfg<1>::CPS);
        c.S = ws ? cc_splits(d, ws_bytes, &c.per_split) : 1;
        if (c.S == 1) c.per_split = c.nstages;
        const bool fold = c.S > 1 && tickets;        // combine in the conv launch
        if (c.S > 1 && !tickets) c.tickets = nullptr;
        const dim3 grid((c.M + CC_BM - 1) / CC_BM, (d->cout + CC_BN - 1) / CC_BN, c.S);
        CcArgs cl = c;
        if (c.S > 1 && !fold) cl.S = -c.S;            // slabs only; k_conv_reduce combines
        launch_cc(cl, grid, st);
        if (c.S > 1 && !fold) {
            const int64_t total = (int64_t)c.M * d->cout;
            hipLaunchKernelGGL(k_conv_reduce, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, c.S, total,
                               d->cout, c.HW, c.part, bias, residual, y);
        }
        RDQ_CHECK(hipGetLastError());
        return 0;
    }
    IgArgs a{};
    a.d = *d; a.x = x; a.x2 = x2; a.w = w; a.bias = bias; a.res = residual; a.y = y;
    a.part = static_cast<float *>(ws);
    a.K = (d->cin1 + d->cin2) * d->kh * d->kw;
    a.HW = d->H * d->W;
    a.M = d->B * a.HW;
    a.nsteps = (a.K + IG_BK - 1) / IG_BK;
    a.S = ws ? ig_splits(d, ws_bytes, &a.per_split) : 1;
    if (a.S == 1) a.per_split = a.nsteps;
    const dim3 grid((a.M + IG_BM - 1) / IG_BM, (d->cout + IG_BN - 1) / IG_BN, a.S);
    const bool sq = d->kh == d->kw;
    if (sq && d->kh == 3) launch_conv_ig<3>(grid, st, a);
    else if (sq && d->kh == 1) launch_conv_ig<1>(grid, st, a);
    else if (sq && d->kh == 7) launch_conv_ig<7>(grid, st, a);
    else launch_conv_ig<0>(grid, st, a);
    if (a.S > 1) {
        const int64_t total = (int64_t)a.M * d->cout;
        hipLaunchKernelGGL(k_conv_reduce, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, a.S, total, d->cout,
                           a.HW, a.part, bias, residual, y);
    }
    RDQ_CHECK(hipGetLastError());
    return 0;
}

size_t rdq_conv2d_gn_ws_bytes(const rdq_conv_desc *d, int32_t G)
{
    if (!d || !cc_ok(d) || G < 1 || d->cout % G || d->H * d->W < CC_BM) return 0;
    const int cpg = d->cout / G;
    if (cpg < 8 || cpg > CC_BN || CC_BN % cpg) return 0;
    const size_t M = (size_t)d->B * d->H * d->W, mt = (M + CC_BM - 1) / CC_BM;
    return rdq_conv2d_ws_bytes(d) + M * d->cout * sizeof(float) + mt * G * 4 * sizeof(double);
}

// arguments of the conv of rdq_conv2d_gn_silu (output and statistics in ws); false: not applicable
static bool gn_conv_args(CcArgs &c, const rdq_conv_desc *d, const float *x, const float *x2, const float *w,
                         const float *bias, int32_t G, void *ws, size_t ws_bytes, uint32_t *tickets)
{
    const size_t need = rdq_conv2d_gn_ws_bytes(d, G);
    if (!need || !x || !w || !ws || ws_bytes < need || (d->cin2 > 0 && !x2 && d->in_mode == RDQ_IN_PLAIN))
        return false;
    if (d->in_mode == RDQ_IN_UNSHUFFLE2 && (d->cin1 % 4 != 0 || d->cin2 != 0)) return false;
    if (d->in_mode == RDQ_IN_UPSAMPLE2 && ((d->H | d->W) & 1 || d->cin2 != 0)) return false;
    const size_t M = (size_t)d->B * d->H * d->W;
    const size_t slabs = rdq_conv2d_ws_bytes(d);
    float *h = reinterpret_cast<float *>(static_cast<char *>(ws) + slabs);
    c = CcArgs{};
    c.d = *d; c.x = x; c.x2 = x2; c.w = w; c.bias = bias; c.res = nullptr; c.y = h;
    c.part = static_cast<float *>(ws);
    c.tickets = tickets;
    c.gnp = reinterpret_cast<double *>(h + M * d->cout);
    c.G = G;
    c.K = (d->cin1 + d->cin2) * d->kh * d->kw;
    c.HW = d->H * d->W;
    c.M = (int)M;
    cc_extents(c, d);
    c.nstages = (d->cin1 + d->cin2) / (d->kh == 3 ? CcCfg<9>::CPS : CcCfg<1>::CPS);
    c.S = (slabs && tickets) ? cc_splits(d, slabs, &c.per_split) : 1;   // statistics need the in-launch combine
    if (c.S == 1) c.per_split = c.nstages;
    return true;
}

// the conv of a gn_conv_args Block on the fp32 halo-staged kernel when it applies (a 256-pixel tile
// then spans at most two samples, as the statistics' slots assume); true: launched, bm = C3_BM
static bool conv3f_gn(const CcArgs &c, const rdq_conv_desc *d, int32_t G, hipStream_t st)
{
    if (!conv3f_ok(d) || d->H * d->W < C3_BM) return false;
    launch_conv3_f32(d, c.x, c.x2, c.w, c.bias, nullptr, c.y, c.gnp, G, st);
    return true;
}

int rdq_conv2d_gn_silu(const rdq_conv_desc *d, const float *x, const float *x2, const float *w, const float *bias,
                       int32_t G, float eps, const float *gamma, const float *beta, const float *scale_shift,
                       const float *post_residual, float *y, void *ws, size_t ws_bytes, uint32_t *tickets,
                       hipStream_t st)
{
    CcArgs c;
    if (!y || !gamma || !beta || !gn_conv_args(c, d, x, x2, w, bias, G, ws, ws_bytes, tickets)) return RDQ_E_INVALID;
    float *h = c.y;
    double *gnp = c.gnp;
    const dim3 grid((c.M + CC_BM - 1) / CC_BM, (d->cout + CC_BN - 1) / CC_BN, c.S);
    const int bm = conv3f_gn(c, d, G, st) ? C3_BM : CC_BM;    // launched there, or here:
    if (bm == CC_BM) launch_cc(c, grid, st);
    const int C = d->cout, HW = c.HW;
    int nch = 0;
    bool gn4 = false;
    const int gxa = gn_grid(d->B, C, G, HW, &nch, &gn4);
    LAUNCH_GN_T(dim3(gxa, d->B * G), st, C, HW, G, nch, h, gamma, beta,
                       scale_shift, gnp, eps, post_residual, y, bm);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

static rdq_conv_desc shortcut_desc(const rdq_conv_desc *d, int cout_s)
{
    rdq_conv_desc ds = *d;
    ds.cout = cout_s; ds.kh = ds.kw = 1; ds.pad = 0;
    return ds;
}

size_t rdq_conv2d_gn_sc_ws_bytes(const rdq_conv_desc *d, int32_t G, int32_t cout_s)
{
    const size_t a = rdq_conv2d_gn_ws_bytes(d, G);
    if (!a || cout_s < 1 || d->in_mode != RDQ_IN_PLAIN || d->kh != 3) return 0;
    const rdq_conv_desc ds = shortcut_desc(d, cout_s);
    if (!cc_ok(&ds)) return 0;
    return a + rdq_conv2d_ws_bytes(&ds);
}

size_t rdq_conv2d_gn_sc_tickets(const rdq_conv_desc *d, int32_t cout_s)
{
    const rdq_conv_desc ds = shortcut_desc(d, cout_s);
    return rdq_conv2d_tickets(d) + rdq_conv2d_tickets(&ds);
}

int rdq_conv2d_gn_silu_sc(const rdq_conv_desc *d, const float *x, const float *x2, const float *w, const float *bias,
                          int32_t G, float eps, const float *gamma, const float *beta, const float *scale_shift,
                          float *y, int32_t cout_s, const float *w_s, const float *b_s, float *y_s, void *ws,
                          size_t ws_bytes, uint32_t *tickets, hipStream_t st)
{
    const size_t need = rdq_conv2d_gn_sc_ws_bytes(d, G, cout_s);
    if (!need || !x || !w || !y || !gamma || !beta || !w_s || !y_s || !ws || ws_bytes < need ||
        (d->cin2 > 0 && !x2))
        return RDQ_E_INVALID;
    const rdq_conv_desc ds = shortcut_desc(d, cout_s);
    const size_t M = (size_t)d->B * d->H * d->W;
    const size_t wa = rdq_conv2d_gn_ws_bytes(d, G), slabs = rdq_conv2d_ws_bytes(d), slabs_s = rdq_conv2d_ws_bytes(&ds);
    float *h = reinterpret_cast<float *>(static_cast<char *>(ws) + slabs);
    // block1's conv: exactly the arguments of rdq_conv2d_gn_silu
    CcArgs c{};
    c.d = *d; c.x = x; c.x2 = x2; c.w = w; c.bias = bias; c.res = nullptr; c.y = h;
    c.part = static_cast<float *>(ws);
    c.tickets = tickets;
    c.gnp = reinterpret_cast<double *>(h + M * d->cout);
    c.G = G;
    c.K = (d->cin1 + d->cin2) * 9;
    c.HW = d->H * d->W;
    c.M = (int)M;
    cc_extents(c, d);
    c.nstages = (d->cin1 + d->cin2) / CcCfg<9>::CPS;
    c.S = (slabs && tickets) ? cc_splits(d, slabs, &c.per_split) : 1;
    if (c.S == 1) c.per_split = c.nstages;
    // the shortcut: exactly the arguments of rdq_conv2d (split-K combined in the launch)
    CcArgs e{};
    e.d = ds; e.x = x; e.x2 = x2; e.w = w_s; e.bias = b_s; e.res = nullptr; e.y = y_s;
    e.part = reinterpret_cast<float *>(static_cast<char *>(ws) + wa);
    e.tickets = tickets ? tickets + rdq_conv2d_tickets(d) : nullptr;
    e.K = ds.cin1 + ds.cin2;
    e.HW = c.HW;
    e.M = c.M;
    cc_extents(e, &ds);
    e.nstages = (ds.cin1 + ds.cin2) / CcCfg<1>::CPS;
    e.S = (slabs_s && tickets) ? cc_splits(&ds, slabs_s, &e.per_split) : 1;
    if (e.S == 1) e.per_split = e.nstages;
    const int gy_a = (d->cout + CC_BN - 1) / CC_BN, gy_b = (cout_s + CC_BN - 1) / CC_BN;
    int bm = CC_BM;
    if (conv3f_gn(c, d, G, st)) {     // the 3x3 on the halo-staged kernel, the shortcut on its own
        bm = C3_BM;
        launch_cc(e, dim3((e.M + CC_BM - 1) / CC_BM, gy_b, e.S), st);
    } else {
        const dim3 grid((c.M + CC_BM - 1) / CC_BM, gy_a + gy_b, std::max(c.S, e.S));
        hipLaunchKernelGGL(k_conv_cc_pair, grid, dim3(256), 0, st, c, e, gy_a);
    }
    const int C = d->cout, HW = c.HW;
    int nch = 0;
    bool gn4 = false;
    const int gxa = gn_grid(d->B, C, G, HW, &nch, &gn4);
    LAUNCH_GN_T(dim3(gxa, d->B * G), st, C, HW, G, nch, h, gamma, beta,
                       scale_shift, c.gnp, eps, nullptr, y, bm);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

int rdq_conv2d_gn_silu_lsm(const rdq_conv_desc *d, const float *x, const float *x2, const float *w, const float *bias,
                           int32_t G, float eps, const float *gamma, const float *beta, const float *post_residual,
                           float *y, void *ws, size_t ws_bytes, uint32_t *tickets, int32_t in, const float *temb,
                           int32_t n, const float *const *lw, const float *const *lb, const int32_t *lout,
                           float *const *ly, int32_t ss_index, hipStream_t st)
{
    CcArgs c;
    if (!y || !gamma || !beta || !temb || in < 1 || n < 1 || n > LM_MAX || !lw || !lout || !ly ||
        ss_index >= n || d->in_mode != RDQ_IN_PLAIN || !gn_conv_args(c, d, x, x2, w, bias, G, ws, ws_bytes, tickets))
        return RDQ_E_INVALID;
    LinMulti L{};
    L.n = n;
    L.start[0] = 0;
    for (int j = 0; j < n; ++j) {
        if (!lw[j] || !ly[j] || lout[j] < 1) return RDQ_E_INVALID;
        L.w[j] = lw[j];
        L.b[j] = lb ? lb[j] : nullptr;
        L.y[j] = ly[j];
        L.out[j] = lout[j];
        L.start[j + 1] = L.start[j] + lout[j];
    }
    if (ss_index >= 0 && lout[ss_index] != 2 * d->cout) return RDQ_E_INVALID;
    const int per_b = (L.start[n] + 4 * LSM_RPW - 1) / (4 * LSM_RPW), nlsm = per_b * d->B;
    const dim3 grid(nlsm + (c.M + CC_BM - 1) / CC_BM, (d->cout + CC_BN - 1) / CC_BN, c.S);
    if (d->kh == 3)
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_conv_cc_lsm<9, RDQ_IN_PLAIN>), grid, dim3(256), 0, st, c, L, in, temb,
                           nlsm, per_b);
    else
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_conv_cc_lsm<1, RDQ_IN_PLAIN>), grid, dim3(256), 0, st, c, L, in, temb,
                           nlsm, per_b);
    const int C = d->cout, HW = c.HW;
    int nch = 0;
    bool gn4 = false;
    const int gxa = gn_grid(d->B, C, G, HW, &nch, &gn4);
    LAUNCH_GN_T(dim3(gxa, d->B * G), st, C, HW, G, nch, c.y, gamma, beta,
                       ss_index >= 0 ? ly[ss_index] : nullptr, c.gnp, eps, post_residual, y);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

int rdq_conv2d_gn_silu_out(const rdq_conv_desc *d, const float *x, const float *x2, const float *w, const float *bias,
                           int32_t G, float eps, const float *gamma, const float *beta, const float *scale_shift,
                           const float *post_residual, int32_t nf, const float *wf, const float *bf, float *yf,
                           void *ws, size_t ws_bytes, uint32_t *tickets, hipStream_t st)
{
    CcArgs c;
    if (!yf || !wf || !gamma || !beta || nf < 1 || nf > GO_MAXF || d->cout % 4 || G > 64 ||
        !gn_conv_args(c, d, x, x2, w, bias, G, ws, ws_bytes, tickets))
        return RDQ_E_INVALID;
    const dim3 grid((c.M + CC_BM - 1) / CC_BM, (d->cout + CC_BN - 1) / CC_BN, c.S);
    const int bm = conv3f_gn(c, d, G, st) ? C3_BM : CC_BM;    // launched there, or here:
    if (bm == CC_BM) launch_cc(c, grid, st);
    const int HW = c.HW;
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_gn_apply_out<float>), dim3((HW + 63) / 64, d->B), dim3(64 * GO_NW), 0, st, d->cout, HW, G, c.y, gamma, beta,
                       scale_shift, c.gnp, eps, post_residual, nf, wf, bf, yf, bm);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

int rdq_unet_head(const rdq_conv_desc *d, const float *x, const float *w, const float *bias, float *y, int32_t dim,
                  float theta, const int64_t *t, const float *w1, const float *b1, int32_t hid, const float *w2,
                  const float *b2, int32_t out, float *temb, hipStream_t st)
{
    if (!d || !x || !w || !y || !t || !w1 || !b1 || !w2 || !b2 || !temb || d->B < 1 || d->cin1 < 1 ||
        d->cin2 != 0 || d->in_mode != RDQ_IN_PLAIN || d->cout < 1 || d->cout > IG_BN || d->kh != d->kw ||
        (d->kh != 7 && d->kh != 3) || d->pad < 0 || d->H < 1 || d->W < 1 || cc_ok(d))
        return RDQ_E_INVALID;
    if (dim < 4 || dim % 2 || hid < 1 || out < 1 || dim + hid > IG_SMEM) return RDQ_E_INVALID;
    IgArgs a{};
    a.d = *d; a.x = x; a.x2 = nullptr; a.w = w; a.bias = bias; a.res = nullptr; a.y = y;
    a.K = d->cin1 * d->kh * d->kw;
    a.HW = d->H * d->W;
    a.M = d->B * a.HW;
    a.nsteps = (a.K + IG_BK - 1) / IG_BK;
    int per = 0;
    if (ig_splits(d, (size_t)-1 / 2, &per) != 1) return RDQ_E_INVALID;    // rdq_conv2d would split K
    a.S = 1;
    a.per_split = a.nsteps;
    const int half = dim / 2;
    const float emb = (float)(std::log((double)theta) / (double)(half - 1));   // python float math
    const TmArgs m{dim, hid, out, -emb, t, w1, b1, w2, b2, temb};
    const int gxc = (a.M + IG_BM - 1) / IG_BM, tm_x = (out + TM_ROWS - 1) / TM_ROWS;
    const dim3 grid(gxc + tm_x * d->B);
    if (d->kh == 7) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_unet_head<7>), grid, dim3(256), 0, st, a, gxc, m, tm_x);
    else hipLaunchKernelGGL(HIP_KERNEL_NAME(k_unet_head<3>), grid, dim3(256), 0, st, a, gxc, m, tm_x);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

int rdq_conv2d_rms(const rdq_conv_desc *d, const float *x, const float *g, const float *w, const float *bias,
                   const float *residual, float *y, void *ws, size_t ws_bytes, uint32_t *tickets, hipStream_t st)
{
    if (!d || !x || !g || !w || !y || !cc_ok(d) || d->kh != 1 || d->in_mode != RDQ_IN_PLAIN || d->cin2 != 0 ||
        d->cin1 > 2048)
        return RDQ_E_INVALID;
    CcArgs c{};
    c.d = *d; c.x = x; c.x2 = nullptr; c.w = w; c.bias = bias; c.res = residual; c.y = y;
    c.part = static_cast<float *>(ws);
    c.tickets = tickets;
    c.rms_g = g;
    c.K = d->cin1;
    c.HW = d->H * d->W;
    c.M = d->B * c.HW;
    cc_extents(c, d);
    c.nstages = d->cin1 / CcCfg<1>::CPS;
    c.S = (ws && tickets) ? cc_splits(d, ws_bytes, &c.per_split) : 1;
    if (c.S == 1) c.per_split = c.nstages;
    const dim3 grid((c.M + CC_BM - 1) / CC_BM, (d->cout + CC_BN - 1) / CC_BN, c.S);
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_conv_cc<1, RDQ_IN_PLAIN, true>), grid, dim3(256), 0, st, c);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

size_t rdq_conv2d_bf16_wpack_bytes(const rdq_conv_desc *d)
{
    if (!conv_desc_ok(d)) return 0;
    return (size_t)d->cout * d->kh * d->kw * bf_cinp(d) * sizeof(__bf16);
}

int rdq_conv2d_bf16_pack(const rdq_conv_desc *d, const float *w, void *wp, hipStream_t st)
{
    if (!conv_desc_ok(d) || !w || !wp) return RDQ_E_INVALID;
    const int taps = d->kh * d->kw, cinp = bf_cinp(d);
    const int64_t n = (int64_t)d->cout * taps * cinp;
    const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_pack_w_bf16, dim3(blocks), dim3(256), 0, st, d->cout, d->cin1 + d->cin2, taps, cinp, w,
                       static_cast<__bf16 *>(wp));
    RDQ_CHECK(hipGetLastError());
    return 0;
}

size_t rdq_conv2d_bf16_ws_bytes(const rdq_conv_desc *d)
{
    if (!conv_desc_ok(d)) return 0;
    const int BN = d->cout >= 128 ? 128 : 64;
    int per = 0;
    const int S = bf_splits(d, BN, d->kh * d->kw * bf_cinp(d) / BF_BK, (size_t)-1 / 2, &per);
    return S > 1 ? (size_t)S * d->B * d->H * d->W * d->cout * sizeof(float) : 0;
}

static std::atomic<int> g_bf16_per_tap{0};   // RDQ_UNET_OPT_BF16_PER_TAP

int rdq_unet_set_option(int32_t option, int32_t value)
{
    std::atomic<int> *opt = nullptr;
    switch (option) {
    case RDQ_UNET_OPT_BF16_PER_TAP: opt = &g_bf16_per_tap; value = value != 0; break;
    case RDQ_UNET_OPT_CONV3_MIN_TILES: if (value < 1) return RDQ_E_INVALID; opt = &C3_MIN_TILES; break;
    case RDQ_UNET_OPT_BF16_RAW: opt = &C3_BF16_RAW; value = value != 0; break;
    case RDQ_UNET_OPT_CONV3F_MIN_TILES: if (value < 0) return RDQ_E_INVALID; opt = &C3F_MIN_TILES; break;
    case RDQ_UNET_OPT_CC_MIN_STAGES: if (value < 1) return RDQ_E_INVALID; opt = &CC_MIN_STAGES; break;
    case RDQ_UNET_OPT_CC_SPLIT2_STAGES: if (value < 1) return RDQ_E_INVALID; opt = &CC_SPLIT2_STAGES; break;
    default: return RDQ_E_INVALID;
    }
    const int old = opt->exchange(value);
    if (old != value) g_opt_gen.fetch_add(1);
    return old;
}

int rdq_unet_options_generation(void) { return g_opt_gen.load(); }

int rdq_conv2d_stem(const rdq_conv_desc *d, const float *x, const float *w, const float *bias, float *y, hipStream_t st)
{
    if (!conv_desc_ok(d) || !x || !w || !y || d->cin1 != 1 || d->cin2 != 0 || d->kh != ST_K || d->kw != ST_K ||
        d->pad != ST_K / 2 || d->cout != ST_C || d->in_mode != RDQ_IN_PLAIN || d->W < 64 || d->W > C3_WMAX ||
        (int64_t)d->B * ST_C * d->H * d->W >= ((int64_t)1 << 31))
        return RDQ_E_INVALID;
    if (d->W % 2 == 0)
        hipLaunchKernelGGL(k_stem7x2, dim3((d->H * d->W + 511) / 512, d->B), dim3(256), 0, st, d->H, d->W, x, w, bias, y);
    else
        hipLaunchKernelGGL(k_stem7, dim3((d->H * d->W + 255) / 256, d->B), dim3(256), 0, st, d->H, d->W, x, w, bias, y);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

int rdq_conv2d_bf16(const rdq_conv_desc *d, const float *x, const float *x2, const void *wp, const float *bias,
                    const float *residual, float *y, void *ws, size_t ws_bytes, hipStream_t st)
{
    if (!conv_desc_ok(d) || !x || !wp || !y || (d->cin2 > 0 && !x2 && d->in_mode == RDQ_IN_PLAIN))
        return RDQ_E_INVALID;
    if (conv3_ok(d) && !g_bf16_per_tap) {
        C3Args c{};
        c.d = *d; c.x = x; c.x2 = x2; c.w = static_cast<const __bf16 *>(wp); c.bias = bias; c.res = residual; c.y = y;
        c.cinp = bf_cinp(d);
        c.K = 9 * c.cinp;
        c.HW = d->H * d->W;
        c.M = d->B * c.HW;
        c.R = C3_BM + 2 * d->W + 2;
        c.cch = c.cinp / BF_BK;
        c.plane = d->in_mode == RDQ_IN_UPSAMPLE2 ? c.HW / 4 : c.HW;
        const dim3 grid((c.M + C3_BM - 1) / C3_BM, d->cout / C3_BN);
        if (d->in_mode == RDQ_IN_UPSAMPLE2)
            hipLaunchKernelGGL(HIP_KERNEL_NAME(k_conv3_bf16<RDQ_IN_UPSAMPLE2>), grid, dim3(256), 0, st, c);
        else
            hipLaunchKernelGGL(HIP_KERNEL_NAME(k_conv3_bf16<RDQ_IN_PLAIN>), grid, dim3(256), 0, st, c);
        RDQ_CHECK(hipGetLastError());
        return 0;
    }
    BfArgs a{};
    a.d = *d; a.x = x; a.x2 = x2; a.w = static_cast<const __bf16 *>(wp); a.bias = bias; a.res = residual; a.y = y;
    a.part = static_cast<float *>(ws);
    a.cinp = bf_cinp(d);
    a.K = d->kh * d->kw * a.cinp;
    a.HW = d->H * d->W;
    a.M = d->B * a.HW;
    a.nsteps = a.K / BF_BK;
    const int NB = d->cout >= 128 ? 4 : 2;
    a.S = ws ? bf_splits(d, 32 * NB, a.nsteps, ws_bytes, &a.per_split) : 1;
    if (a.S == 1) a.per_split = a.nsteps;
    const dim3 grid((a.M + BF_BM - 1) / BF_BM, (d->cout + 32 * NB - 1) / (32 * NB), a.S);
    if (NB == 4) launch_conv_bf16<4>(grid, st, a);
    else launch_conv_bf16<2>(grid, st, a);
    if (a.S > 1) {
        const int64_t total = (int64_t)a.M * d->cout;
        hipLaunchKernelGGL(k_conv_reduce, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, a.S, total, d->cout,
                           a.HW, a.part, bias, residual, y);
    }
    RDQ_CHECK(hipGetLastError());
    return 0;
}

size_t rdq_conv2d_bf16_gn_ws_bytes(const rdq_conv_desc *d, int32_t G)
{
    if (!d || !conv_desc_ok(d) || !conv3_ok(d) || G < 1 || d->cout % G || d->H * d->W < C3_BM) return 0;
    const int cpg = d->cout / G;
    if (cpg < 8 || cpg > C3_BN || C3_BN % cpg) return 0;
    const size_t M = (size_t)d->B * d->H * d->W, mt = (M + C3_BM - 1) / C3_BM;
    return M * d->cout * sizeof(float) + mt * G * 4 * sizeof(double);
}

int rdq_conv2d_bf16_gn_silu(const rdq_conv_desc *d, const float *x, const float *x2, const void *wp, const float *bias,
                            int32_t G, float eps, const float *gamma, const float *beta, const float *scale_shift,
                            const float *post_residual, float *y, void *ws, size_t ws_bytes, hipStream_t st);

// conv3x3_bf16 + GroupNorm statistics in its epilogue (as rdq_conv2d_bf16_gn_silu), conv output in ws
static bool bf16_gn_conv(const rdq_conv_desc *d, const float *x, const float *x2, const void *wp, const float *bias,
                         int32_t G, void *ws, size_t ws_bytes, C3Args &c, hipStream_t st, const void *x8 = nullptr)
{
    const size_t need = rdq_conv2d_bf16_gn_ws_bytes(d, G);
    if (!need || !(x || x8) || !wp || !ws || ws_bytes < need || (d->cin2 > 0 && !x2 && d->in_mode == RDQ_IN_PLAIN))
        return false;
    // packed bf16 octet input: plain mode, one input tensor, channel count a multiple of the 32-deep chunk
    if (x8 && (d->in_mode != RDQ_IN_PLAIN || d->cin2 != 0 || d->cin1 % BF_BK ||
               (int64_t)d->B * d->cin1 * d->H * d->W >= ((int64_t)1 << 32)))
        return false;
    const size_t M = (size_t)d->B * d->H * d->W;
    float *h = static_cast<float *>(ws);
    c = C3Args{};
    c.d = *d; c.x = x; c.x2 = x2; c.w = static_cast<const __bf16 *>(wp); c.bias = bias; c.res = nullptr; c.y = h;
    c.yb = C3_BF16_RAW ? reinterpret_cast<__bf16 *>(h) : nullptr;   // raw conv output held as bf16
    c.gnp = reinterpret_cast<double *>(h + M * d->cout);
    c.G = G;
    c.cinp = bf_cinp(d);
    c.K = 9 * c.cinp;
    c.HW = d->H * d->W;
    c.M = (int)M;
    c.R = C3_BM + 2 * d->W + 2;
    c.cch = c.cinp / BF_BK;
    c.plane = d->in_mode == RDQ_IN_UPSAMPLE2 ? c.HW / 4 : c.HW;
    c.x8 = static_cast<const __bf16 *>(x8);
    const dim3 grid((c.M + C3_BM - 1) / C3_BM, d->cout / C3_BN);
    if (x8)
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_conv3_bf16<RDQ_IN_PLAIN, true>), grid, dim3(256), 0, st, c);
    else if (d->in_mode == RDQ_IN_UPSAMPLE2)
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_conv3_bf16<RDQ_IN_UPSAMPLE2>), grid, dim3(256), 0, st, c);
    else
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_conv3_bf16<RDQ_IN_PLAIN>), grid, dim3(256), 0, st, c);
    return true;
}

int rdq_conv2d_bf16_gn_silu8(const rdq_conv_desc *d, const float *x, const float *x2, const void *wp,
                             const float *bias, int32_t G, float eps, const float *gamma, const float *beta,
                             const float *scale_shift, void *y8, void *ws, size_t ws_bytes, hipStream_t st)
{
    C3Args c;
    if (!y8 || !gamma || !beta || d->cout % 8 || (int64_t)d->B * d->cout * d->H * d->W >= ((int64_t)1 << 32) ||
        !bf16_gn_conv(d, x, x2, wp, bias, G, ws, ws_bytes, c, st))
        return RDQ_E_INVALID;
    const int HW = c.HW;
    if (c.yb && HW % 2 == 0)
        hipLaunchKernelGGL(k_gn_apply8x2, dim3((HW + 511) / 512, d->B * G), dim3(256), 0, st,
                           d->cout, HW, G, c.yb, gamma, beta, scale_shift, c.gnp, eps, static_cast<__bf16 *>(y8), C3_BM);
    else if (c.yb)
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_gn_apply8<__bf16>), dim3((HW + 255) / 256, d->B * G), dim3(256), 0, st, d->cout,
                           HW, G, c.yb, gamma, beta, scale_shift, c.gnp, eps, static_cast<__bf16 *>(y8), C3_BM);
    else
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_gn_apply8<float>), dim3((HW + 255) / 256, d->B * G), dim3(256), 0, st, d->cout,
                           HW, G, c.y, gamma, beta, scale_shift, c.gnp, eps, static_cast<__bf16 *>(y8), C3_BM);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

int rdq_conv2d_bf16_gn_silu_x8(const rdq_conv_desc *d, const void *x8, const void *wp, const float *bias, int32_t G,
                               float eps, const float *gamma, const float *beta, const float *scale_shift,
                               const float *post_residual, float *y, void *ws, size_t ws_bytes, hipStream_t st)
{
    C3Args c;
    if (!y || !gamma || !beta || !x8 || !bf16_gn_conv(d, nullptr, nullptr, wp, bias, G, ws, ws_bytes, c, st, x8))
        return RDQ_E_INVALID;
    const int C = d->cout, HW = c.HW;
    int nch = 0;
    bool gn4 = false;
    const int gxa = gn_grid(d->B, C, G, HW, &nch, &gn4);
    if (c.yb)
        LAUNCH_GN_TB(dim3(gxa, d->B * G), st, C, HW, G, nch, c.yb, gamma, beta, scale_shift, c.gnp, eps, post_residual, y,
                     C3_BM);
    else
        LAUNCH_GN_T(dim3(gxa, d->B * G), st, C, HW, G, nch, c.y, gamma, beta, scale_shift, c.gnp, eps, post_residual, y,
                    C3_BM);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

int rdq_conv2d_bf16_gn_silu(const rdq_conv_desc *d, const float *x, const float *x2, const void *wp, const float *bias,
                            int32_t G, float eps, const float *gamma, const float *beta, const float *scale_shift,
                            const float *post_residual, float *y, void *ws, size_t ws_bytes, hipStream_t st)
{
    C3Args c;
    if (!y || !gamma || !beta || !bf16_gn_conv(d, x, x2, wp, bias, G, ws, ws_bytes, c, st)) return RDQ_E_INVALID;
    const int C = d->cout, HW = c.HW;
    int nch = 0;
    bool gn4 = false;
    const int gxa = gn_grid(d->B, C, G, HW, &nch, &gn4);
    if (c.yb)
        LAUNCH_GN_TB(dim3(gxa, d->B * G), st, C, HW, G, nch, c.yb, gamma, beta, scale_shift, c.gnp, eps, post_residual, y,
                     C3_BM);
    else
        LAUNCH_GN_T(dim3(gxa, d->B * G), st, C, HW, G, nch, c.y, gamma, beta, scale_shift, c.gnp, eps, post_residual, y,
                    C3_BM);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

int rdq_conv2d_bf16_gn_silu_out(const rdq_conv_desc *d, const float *x, const float *x2, const void *wp,
                                const float *bias, int32_t G, float eps, const float *gamma, const float *beta,
                                const float *scale_shift, const float *post_residual, int32_t nf, const float *wf,
                                const float *bf, float *yf, void *ws, size_t ws_bytes, hipStream_t st)
{
    C3Args c;
    if (!yf || !wf || !gamma || !beta || nf < 1 || nf > GO_MAXF || G > 64 ||
        !bf16_gn_conv(d, x, x2, wp, bias, G, ws, ws_bytes, c, st))
        return RDQ_E_INVALID;
    if (c.yb)
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_gn_apply_out<__bf16>), dim3((c.HW + 63) / 64, d->B), dim3(64 * GO_NW), 0, st,
                           d->cout, c.HW, G, c.yb, gamma, beta, scale_shift, c.gnp, eps, post_residual, nf, wf, bf, yf,
                           C3_BM);
    else
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_gn_apply_out<float>), dim3((c.HW + 63) / 64, d->B), dim3(64 * GO_NW), 0, st,
                           d->cout, c.HW, G, c.y, gamma, beta, scale_shift, c.gnp, eps, post_residual, nf, wf, bf, yf,
                           C3_BM);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

size_t rdq_group_norm_ws_bytes(int32_t B, int32_t C, int32_t HW, int32_t G)
{
    if (B < 1 || C < 1 || HW < 1 || G < 1) return 0;
    const int64_t gsize = (int64_t)(C / G) * HW;
    const int64_t nchunk = (gsize + GN_CHUNK - 1) / GN_CHUNK;
    return (size_t)B * G * nchunk * 2 * sizeof(double) + (size_t)B * G * 2 * sizeof(float);   // + stats
}

int rdq_group_norm_silu(int32_t B, int32_t C, int32_t HW, int32_t G, float eps, const float *x, const float *gamma,
                        const float *beta, const float *ss, float *y, void *ws, hipStream_t st)
{
    if (B < 1 || C < 1 || HW < 1 || G < 1 || C % G || !x || !gamma || !beta || !y || !ws) return RDQ_E_INVALID;
    const int64_t gsize = (int64_t)(C / G) * HW;
    const int nchunk = (int)((gsize + GN_CHUNK - 1) / GN_CHUNK);
    double *part = (double *)ws;
    float *stat = (float *)(part + (size_t)B * G * nchunk * 2);
    hipLaunchKernelGGL(k_gn_partial, dim3(nchunk, B * G), dim3(256), 0, st, x, gsize, nchunk, part);
    int nch = 0;
    const int gxa = gn_grid(B, C, G, HW, &nch);
    const int64_t blocks = (int64_t)gxa * B * G;
    const bool sep = blocks > 4096;                    // a separate statistics pass pays off
    if (sep)
        hipLaunchKernelGGL(k_gn_stats, dim3((B * G + 255) / 256), dim3(256), 0, st, B * G, nchunk, gsize, eps, part, stat);
    LAUNCH_GN(dim3(gxa, B * G), st, C, HW, G, nch, x, gamma, beta, ss,
                       sep ? stat : nullptr, part, nchunk, eps, y);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

int rdq_rmsnorm(int32_t B, int32_t C, int32_t HW, const float *x, const float *g, const float *res, float *y,
                hipStream_t st)
{
    if (B < 1 || C < 1 || HW < 1 || !x || !g || !y) return RDQ_E_INVALID;
    const bool done = HW >= 2048 ? launch_rmsnorm_r<64>(B, C, HW, x, g, res, y, st)
                    : HW >= 256 ? launch_rmsnorm_r<32>(B, C, HW, x, g, res, y, st)
                                : launch_rmsnorm_r<16>(B, C, HW, x, g, res, y, st);
    if (!done) hipLaunchKernelGGL(k_rmsnorm, dim3((HW + 63) / 64, B), dim3(64 * RMS_G), 0, st, C, HW, x, g, res, y);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

int rdq_linear(int32_t B, int32_t in, int32_t out, const float *x, const float *w, const float *bias, int32_t act_in,
               int32_t act_out, float *y, hipStream_t st)
{
    if (B < 1 || in < 1 || out < 1 || !x || !w || !y) return RDQ_E_INVALID;
    hipLaunchKernelGGL(k_linear, dim3((out + 3) / 4, B), dim3(256), 0, st, in, out, x, w, bias, act_in, act_out, y);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

int rdq_sinusoidal_emb(int32_t B, int32_t dim, float theta, const int64_t *t, float *y, hipStream_t st)
{
    if (B < 1 || dim < 4 || dim % 2 || dim > 2048 || !t || !y) return RDQ_E_INVALID;
    const int half = dim / 2;
    const float emb = (float)(std::log((double)theta) / (double)(half - 1));   // python float math
    hipLaunchKernelGGL(k_sinusoidal, dim3(B), dim3(half), 0, st, dim, -emb, t, y);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

int rdq_time_mlp(int32_t B, int32_t dim, float theta, const int64_t *t, const float *w1, const float *b1, int32_t hid,
                 const float *w2, const float *b2, int32_t out, float *y, hipStream_t st)
{
    if (B < 1 || dim < 4 || dim % 2 || hid < 1 || out < 1 || (size_t)(dim + hid) * 4 * TMB > 64 * 1024 ||
        !t || !w1 || !b1 || !w2 || !b2 || !y)
        return RDQ_E_INVALID;
    const int half = dim / 2;
    const float emb = (float)(std::log((double)theta) / (double)(half - 1));   // python float math
    const TmArgs m{dim, hid, out, -emb, t, w1, b1, w2, b2, y};
    if (B > 2 * TMB)
        hipLaunchKernelGGL(k_time_mlp_b, dim3((out + 4 * TMB_RW - 1) / (4 * TMB_RW), (B + TMB - 1) / TMB), dim3(256),
                           TMB * (dim + hid) * sizeof(float), st, m, B);
    else
        hipLaunchKernelGGL(k_time_mlp, dim3((out + TM_ROWS - 1) / TM_ROWS, B), dim3(256), (dim + hid) * sizeof(float),
                           st, m);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

int rdq_linear_silu_multi(int32_t B, int32_t in, const float *x, int32_t n, const float *const *w,
                          const float *const *b, const int32_t *out, float *const *y, hipStream_t st)
{
    if (B < 1 || in < 1 || !x || n < 1 || n > LM_MAX || !w || !out || !y) return RDQ_E_INVALID;
    LinMulti L{};
    L.n = n;
    L.start[0] = 0;
    for (int j = 0; j < n; ++j) {
        if (!w[j] || !y[j] || out[j] < 1) return RDQ_E_INVALID;
        L.w[j] = w[j];
        L.b[j] = b ? b[j] : nullptr;
        L.y[j] = y[j];
        L.out[j] = out[j];
        L.start[j + 1] = L.start[j] + out[j];
    }
    if (B > LSB / 2 && in == 256)
        hipLaunchKernelGGL(k_wdot_silu_b, dim3((L.start[n] + 4 * WDR - 1) / (4 * WDR), (B + 63) / 64), dim3(256), 0, st, B,
                           x, L);
    else if (B > LSB / 2 && in <= 256)
        hipLaunchKernelGGL(k_linear_silu_multi_b, dim3((L.start[n] + 4 * LSR - 1) / (4 * LSR), (B + LSB - 1) / LSB),
                           dim3(256), LSB * in * sizeof(float), st, in, B, x, L);
    else
        hipLaunchKernelGGL(k_linear_silu_multi, dim3((L.start[n] + 3) / 4, B), dim3(256), 0, st, in, x, L);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

static int la_chunks(int n, int nmem) { return (n + nmem + LA_CH - 1) / LA_CH; }

size_t rdq_linear_attention_ws_bytes(int32_t B, int32_t heads, int32_t dh, int32_t n, int32_t nmem)
{
    if (B < 1 || heads < 1 || dh < 1 || n < 1 || nmem < 0) return 0;
    const size_t nch = la_chunks(n, nmem);
    return (nch * B * heads * dh * 2 + (nch + 1) * B * heads * dh * dh) * sizeof(float);
}

int rdq_linear_attention(int32_t B, int32_t heads, int32_t dh, int32_t n, int32_t nmem, float scale, const float *qkv,
                         const float *mem_kv, float *out, void *ws, hipStream_t st)
{
    if (B < 1 || heads < 1 || dh < 1 || dh > 32 || n < 1 || nmem < 0 || !qkv || !mem_kv || !out || !ws)
        return RDQ_E_INVALID;
    const int nch = la_chunks(n, nmem);
    float *pstat = (float *)ws;
    float *part = pstat + (size_t)nch * B * heads * dh * 2;
    float *ctx = part + (size_t)nch * B * heads * dh * dh;
    hipLaunchKernelGGL(k_la_ctx, dim3(nch, heads, B), dim3(256), 0, st, heads, dh, n, nmem, qkv, mem_kv, part, pstat);
    const int bhdd = B * heads * dh * dh;
    hipLaunchKernelGGL(k_la_reduce, dim3((bhdd + 255) / 256), dim3(256), 0, st, bhdd, dh, nch, pstat, part, ctx);
    hipLaunchKernelGGL(k_la_out, dim3((n + 63) / 64, heads, B), dim3(256), 0, st, heads, dh, n, scale, qkv, ctx,
                       out);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

int rdq_linear_attention_block(int32_t B, int32_t heads, int32_t dh, int32_t n, int32_t nmem, float scale,
                               const float *qkv, const float *mem_kv, int32_t dim, const float *w_out,
                               const float *b_out, const float *g_out, const float *res, float *y, void *ws,
                               hipStream_t st)
{
    if (B < 1 || heads != 4 || dh != 32 || n < 1 || nmem < 0 || !qkv || !mem_kv || !w_out || !g_out ||
        !y || !ws || (dim != 64 && dim != 128 && dim != 256))
        return RDQ_E_INVALID;
    const int nch = la_chunks(n, nmem);
    float *pstat = (float *)ws;
    float *part = pstat + (size_t)nch * B * heads * dh * 2;
    float *ctx = part + (size_t)nch * B * heads * dh * dh;
    hipLaunchKernelGGL(k_la_ctx, dim3(nch, heads, B), dim3(256), 0, st, heads, dh, n, nmem, qkv, mem_kv, part, pstat);
    int fold = nch;
    const float *src = part;
    if (nch > LAO_MAXCH) {          // many chunks (72 x 72): the combine keeps its own launch
        const int bhdd = B * heads * dh * dh;
        hipLaunchKernelGGL(k_la_reduce, dim3((bhdd + 255) / 256), dim3(256), 0, st, bhdd, dh, nch, pstat, part, ctx);
        fold = 0;
        src = ctx;
    }
    if (dim == 64) launch_la_out_proj<64>(B, heads, n, fold, scale, qkv, pstat, src, w_out, b_out, g_out, res, y, st);
    else if (dim == 128) launch_la_out_proj<128>(B, heads, n, fold, scale, qkv, pstat, src, w_out, b_out, g_out, res, y, st);
    else launch_la_out_proj<256>(B, heads, n, fold, scale, qkv, pstat, src, w_out, b_out, g_out, res, y, st);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

// rdq_linear_attention_bf16: pixel chunks of nsub 64-pixel tiles, about 2048 workgroups per launch
static void lab_split(int B, int n, int *nsub, int *nch)
{
    const int tiles = (n + LB_PX - 1) / LB_PX;
    int s = (int)std::min<int64_t>(16, std::max<int64_t>(2, ((int64_t)tiles * B + 2047) / 2048));
    s = std::min(s, tiles);
    *nsub = s;
    *nch = (tiles + s - 1) / s;
}

size_t rdq_linear_attention_bf16_ws_bytes(int32_t B, int32_t dim, int32_t n)
{
    if (B < 1 || n < 1 || (dim != 64 && dim != 128)) return 0;
    int nsub, nch;
    lab_split(B, n, &nsub, &nch);
    return (size_t)B * nch * LB_PART * sizeof(float);
}

int rdq_linear_attention_bf16(int32_t B, int32_t dim, int32_t n, int32_t nmem, float scale, const float *x,
                              const float *g_in, const void *wqkv, const float *mem_kv, const void *wout,
                              const float *b_out, const float *g_out, float *y, void *ws, size_t ws_bytes,
                              hipStream_t st)
{
    if (B < 1 || n < 1 || nmem < 0 || (dim != 64 && dim != 128) || !x || !g_in || !wqkv ||
        (nmem > 0 && !mem_kv) || !wout || !g_out || !y || !ws || y == x)
        return RDQ_E_INVALID;
    if ((int64_t)B * dim * n >= ((int64_t)1 << 31) || ws_bytes < rdq_linear_attention_bf16_ws_bytes(B, dim, n))
        return RDQ_E_INVALID;
    LabArgs a{};
    a.x = x; a.g_in = g_in; a.mem = mem_kv; a.b_out = b_out; a.g_out = g_out;
    a.wqkv = static_cast<const __bf16 *>(wqkv); a.wout = static_cast<const __bf16 *>(wout);
    a.part = static_cast<float *>(ws); a.y = y;
    a.n = n; a.nmem = nmem; a.scale = scale;
    lab_split(B, n, &a.nsub, &a.nch);
    const dim3 grid(a.nch, B);
    if (dim == 64) {
        hipLaunchKernelGGL(k_lab_kv<64>, grid, dim3(256), 0, st, a);
        hipLaunchKernelGGL(k_lab_out<64>, grid, dim3(256), 0, st, a);
    } else {
        hipLaunchKernelGGL(k_lab_kv<128>, grid, dim3(256), 0, st, a);
        hipLaunchKernelGGL(k_lab_out<128>, grid, dim3(256), 0, st, a);
    }
    RDQ_CHECK(hipGetLastError());
    return 0;
}

// the fp32 form: WGs for about 1024 subtiles (small batches: the combine reads every chunk's partials)
static void lab_split32(int B, int n, int *nsub, int *nch)
{
    const int tiles = (n + LB_PX - 1) / LB_PX;
    int s_ = (int)std::min<int64_t>(16, std::max<int64_t>(1, ((int64_t)tiles * B + 1023) / 1024));
    s_ = std::min(s_, tiles);
    *nsub = s_;
    *nch = (tiles + s_ - 1) / s_;
}

size_t rdq_linear_attention_f32_ws_bytes(int32_t B, int32_t dim, int32_t n)
{
    if (B < 1 || n < 1 || (dim != 64 && dim != 128)) return 0;
    int nsub, nch;
    lab_split32(B, n, &nsub, &nch);
    return (size_t)B * nch * LB_PART * sizeof(float);
}

int rdq_linear_attention_f32(int32_t B, int32_t dim, int32_t n, int32_t nmem, float scale, const float *x,
                             const float *g_in, const float *wqkv, const float *mem_kv, const float *wout,
                             const float *b_out, const float *g_out, float *y, void *ws, size_t ws_bytes,
                             hipStream_t st)
{
    if (B < 1 || n < 1 || nmem < 0 || (dim != 64 && dim != 128) || !x || !g_in || !wqkv ||
        (nmem > 0 && !mem_kv) || !wout || !g_out || !y || !ws || y == x)
        return RDQ_E_INVALID;
    if ((int64_t)B * dim * n >= ((int64_t)1 << 31) || ws_bytes < rdq_linear_attention_f32_ws_bytes(B, dim, n))
        return RDQ_E_INVALID;
    LabArgs a{};
    a.x = x; a.g_in = g_in; a.mem = mem_kv; a.b_out = b_out; a.g_out = g_out;
    a.wqkv32 = wqkv; a.wout32 = wout;
    a.part = static_cast<float *>(ws); a.y = y;
    a.n = n; a.nmem = nmem; a.scale = scale;
    lab_split32(B, n, &a.nsub, &a.nch);
    const dim3 grid(a.nch, B);
    if (dim == 64) {
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_lab_kv<64, true>), grid, dim3(256), 0, st, a);
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_lab_out<64, true>), grid, dim3(256), 0, st, a);
    } else {
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_lab_kv<128, true>), grid, dim3(256), 0, st, a);
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_lab_out<128, true>), grid, dim3(256), 0, st, a);
    }
    RDQ_CHECK(hipGetLastError());
    return 0;
}

int rdq_full_attention(int32_t B, int32_t heads, int32_t dh, int32_t n, int32_t nmem, const float *qkv,
                       const float *mem_kv, float *out, hipStream_t st)
{
    if (B < 1 || heads < 1 || dh != 32 || n < 1 || nmem < 0 || !qkv || !mem_kv || !out) return RDQ_E_INVALID;
    const size_t lds = ((size_t)2 * (nmem + n) * (dh + 1) + (size_t)256 * (dh + 3)) * sizeof(float);
    if (lds > 160 * 1024) return RDQ_E_INVALID;
    hipLaunchKernelGGL(k_full_attn<32>, dim3(heads, B, (n + FA_QB - 1) / FA_QB), dim3(256), lds, st, heads, n, nmem,
                       qkv, mem_kv, out);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

int rdq_red_q_sample(int32_t B, int64_t n, const float *sa, const float *s1a, const int64_t *t, const float *x0,
                     const float *eps, float *xt, hipStream_t st)
{
    if (B < 1 || n < 1 || !sa || !s1a || !t || !x0 || !eps || !xt) return RDQ_E_INVALID;
    hipLaunchKernelGGL(k_red_q_sample, dim3((unsigned)((n + 255) / 256), B), dim3(256), 0, st, n, sa, s1a, t, x0, eps, xt,
                       (int64_t *)nullptr);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

int rdq_red_q_sample_t(int32_t B, int64_t n, const float *sa, const float *s1a, const int64_t *t, const float *x0,
                       const float *eps, float *xt, int64_t *t_out, hipStream_t st)
{
    if (B < 1 || n < 1 || !sa || !s1a || !t || !x0 || !eps || !xt || !t_out) return RDQ_E_INVALID;
    hipLaunchKernelGGL(k_red_q_sample, dim3((unsigned)((n + 255) / 256), B), dim3(256), 0, st, n, sa, s1a, t, x0, eps, xt,
                       t_out);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

int rdq_red_epilogue(int32_t B, int64_t n, const float *sr, const float *srm1, const int64_t *t, const float *xt,
                     const float *eh, const float *eps, float *g, hipStream_t st)
{
    if (B < 1 || n < 1 || !sr || !srm1 || !t || !xt || !eh || !eps || !g) return RDQ_E_INVALID;
    hipLaunchKernelGGL(k_red_epilogue, dim3((unsigned)((n + 255) / 256), B), dim3(256), 0, st, n, sr, srm1, t, xt, eh,
                       eps, g);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

}  // extern "C"
