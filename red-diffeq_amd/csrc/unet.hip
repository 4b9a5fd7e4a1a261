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

#include <cmath>
#include <algorithm>
#include <cstdint>

#include "red_diffeq_unet.h"

namespace {

#define RDQ_CHECK(x)                                   \
    do {                                               \
        hipError_t e_ = (x);                           \
        if (e_ != hipSuccess) return -(int)e_;         \
    } while (0)
#define RDQ_E_INVALID (-10001)

using f32x4 = __attribute__((ext_vector_type(4))) float;

// ------------------------------------------------------------------------------------ conv2d
constexpr int CBM = 64;   // output pixels per workgroup tile
constexpr int CBN = 64;   // output channels per workgroup tile
constexpr int CKC = 16;   // K (= cin*kh*kw) per LDS stage

struct ConvArgs {
    rdq_conv_desc d;
    const float *x, *x2, *w, *bias, *res;
    float *y;
};

__device__ __forceinline__ float conv_in(const ConvArgs &a, int b, int ci, int ih, int iw)
{
    const rdq_conv_desc &d = a.d;
    if (ih < 0 || iw < 0 || ih >= d.H || iw >= d.W) return 0.0f;
    switch (d.in_mode) {
    case RDQ_IN_UPSAMPLE2: {
        const int h2 = d.H >> 1, w2 = d.W >> 1;
        return a.x[(((size_t)b * d.cin1 + ci) * h2 + (ih >> 1)) * w2 + (iw >> 1)];
    }
    case RDQ_IN_UNSHUFFLE2: {
        const int c = ci >> 2, p1 = (ci >> 1) & 1, p2 = ci & 1;
        const int H2 = d.H * 2, W2 = d.W * 2;
        return a.x[(((size_t)b * (d.cin1 >> 2) + c) * H2 + 2 * ih + p1) * W2 + 2 * iw + p2];
    }
    default:
        if (ci < d.cin1) return a.x[(((size_t)b * d.cin1 + ci) * d.H + ih) * d.W + iw];
        return a.x2[(((size_t)b * d.cin2 + (ci - d.cin1)) * d.H + ih) * d.W + iw];
    }
}

// One workgroup = 4 waves = a 64 (pixels) x 64 (channels) output tile; each wave a 32 x 32 quarter
// as 2 x 2 MFMA 16x16 tiles.  MFMA operand maps (gfx950, 16x16x4 f32): lane l supplies
// A[m = l&15][k = l>>4] and B[k = l>>4][n = l&15]; D[m = (l>>4)*4 + r][n = l&15].
__global__ __launch_bounds__(256) void k_conv_mfma(ConvArgs a)
{
    __shared__ float As[CKC][CBM + 4];
    __shared__ float Bs[CKC][CBN + 4];
    const rdq_conv_desc &d = a.d;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid & 1, wn = wid >> 1;
    const int HW = d.H * d.W;
    const int M = d.B * HW, N = d.cout, KK = d.kh * d.kw, K = (d.cin1 + d.cin2) * KK;
    const int m0 = blockIdx.x * CBM, n0 = blockIdx.y * CBN;
    // this thread's gather pixel
    const int am = m0 + (tid & 63);
    const bool mvalid = am < M;
    const int ab = mvalid ? am / HW : 0;
    const int apix = mvalid ? am - ab * HW : 0;
    const int aoh = apix / d.W, aow = apix - aoh * d.W;
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    for (int k0 = 0; k0 < K; k0 += CKC) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int kr = (tid >> 6) + 4 * j, k = k0 + kr;
            float v = 0.0f;
            if (mvalid && k < K) {
                const int ci = k / KK, rem = k - ci * KK;
                const int ky = rem / d.kw, kx = rem - ky * d.kw;
                v = conv_in(a, ab, ci, aoh + ky - d.pad, aow + kx - d.pad);
            }
            As[kr][tid & 63] = v;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int kk = tid & 15, n = (tid >> 4) + 16 * j;
            Bs[kk][n] = (n0 + n < N && k0 + kk < K) ? a.w[(size_t)(n0 + n) * K + k0 + kk] : 0.0f;
        }
        __syncthreads();
#pragma unroll
        for (int ks = 0; ks < CKC / 4; ++ks) {
            const int kr = ks * 4 + (lane >> 4);
            float af[2], bf[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) af[i] = As[kr][wm * 32 + i * 16 + (lane & 15)];
#pragma unroll
            for (int j = 0; j < 2; ++j) bf[j] = Bs[kr][wn * 32 + j * 16 + (lane & 15)];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bf[j], acc[i][j], 0, 0, 0);
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int n = n0 + wn * 32 + j * 16 + (lane & 15);
            if (n >= N) continue;
            const float bv = a.bias ? a.bias[n] : 0.0f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
                if (m >= M) continue;
                const int b = m / HW, pix = m - b * HW;
                const size_t o = ((size_t)b * N + n) * HW + pix;
                float v = acc[i][j][r] + bv;
                if (a.res) v = v + a.res[o];
                a.y[o] = v;
            }
        }
}

// -------------------------------------------------------------------------------- group norm
constexpr int GN_CHUNK = 4096;   // elements per statistics partial

__global__ __launch_bounds__(256) void k_gn_partial(const float *__restrict__ x, int64_t gsize, int nchunk,
                                                    double *__restrict__ part)
{
    const int bg = blockIdx.y, c = blockIdx.x;
    const float *p = x + (size_t)bg * gsize;
    const int64_t e0 = (int64_t)c * GN_CHUNK, e1 = min((int64_t)(c + 1) * GN_CHUNK, gsize);
    double s = 0.0, q = 0.0;
    for (int64_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
        const double v = p[e];
        s += v;
        q += v * v;
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

__global__ __launch_bounds__(256) void k_gn_apply(int C, int HW, int G, float eps, int nchunk,
                                                  const float *__restrict__ x, const float *__restrict__ gamma,
                                                  const float *__restrict__ beta, const float *__restrict__ ss,
                                                  const double *__restrict__ part, float *__restrict__ y)
{
    const int bg = blockIdx.y;                 // (sample, group)
    const int b = bg / G, g = bg - b * G;
    const int cpg = C / G;
    const int64_t gsize = (int64_t)cpg * HW;
    __shared__ float stat[2];
    if (threadIdx.x == 0) {
        double s = 0.0, q = 0.0;
        for (int c = 0; c < nchunk; ++c) { s += part[((size_t)bg * nchunk + c) * 2]; q += part[((size_t)bg * nchunk + c) * 2 + 1]; }
        const double mean = s / (double)gsize;
        double var = q / (double)gsize - mean * mean;
        var = var < 0.0 ? 0.0 : var;
        stat[0] = (float)mean;
        stat[1] = (float)(1.0 / sqrt(var + (double)eps));
    }
    __syncthreads();
    const float mean = stat[0], rstd = stat[1];
    const float *px = x + (size_t)bg * gsize;
    float *py = y + (size_t)bg * gsize;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < gsize; e += (int64_t)gridDim.x * blockDim.x) {
        const int c = g * cpg + (int)(e / HW);
        float v = (px[e] - mean) * rstd;
        v = v * gamma[c] + beta[c];
        if (ss) { const float sc = ss[(size_t)b * 2 * C + c], sh = ss[(size_t)b * 2 * C + C + c]; v = v * (sc + 1.0f) + sh; }
        py[e] = v / (1.0f + expf(-v));   // SiLU
    }
}

// ----------------------------------------------------------------------------------- rmsnorm
__global__ __launch_bounds__(256) void k_rmsnorm(int C, int HW, const float *__restrict__ x,
                                                 const float *__restrict__ g, const float *__restrict__ res,
                                                 float *__restrict__ y)
{
    const int pix = blockIdx.x * blockDim.x + threadIdx.x, b = blockIdx.y;
    if (pix >= HW) return;
    const float *px = x + (size_t)b * C * HW + pix;
    float ssum = 0.0f;
    for (int c = 0; c < C; ++c) { const float v = px[(size_t)c * HW]; ssum += v * v; }
    const float den = fmaxf(sqrtf(ssum), 1e-12f);      // F.normalize: x / max(||x||, eps)
    const float sc = sqrtf((float)C);
    float *py = y + (size_t)b * C * HW + pix;
    const float *pr = res ? res + (size_t)b * C * HW + pix : nullptr;
    for (int c = 0; c < C; ++c) {
        float v = px[(size_t)c * HW] / den;
        v = v * g[c];
        v = v * sc;
        if (pr) v = v + pr[(size_t)c * HW];
        py[(size_t)c * HW] = v;
    }
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

// -------------------------------------------------------------------------- linear attention
// per (b, h, d): softmax statistics of k[d, :] over memory + pixels, then ctx[d][e] = sum_n p v
__global__ __launch_bounds__(256) void k_la_context(int heads, int dh, int n, int nmem, const float *__restrict__ qkv,
                                                    const float *__restrict__ mem, float *__restrict__ ctx)
{
    const int d = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
    const int C = heads * dh;
    const float *krow = qkv + ((size_t)b * 3 * C + C + h * dh + d) * n;
    const float *vbase = qkv + ((size_t)b * 3 * C + 2 * C + h * dh) * n;
    const float *mk = mem + ((size_t)(0 * heads + h) * dh + d) * nmem;   // mem_kv[0][h][d][:]
    const float *mv = mem + (size_t)(1 * heads + h) * dh * nmem;          // mem_kv[1][h][e][:]
    __shared__ float red[256];
    __shared__ float acc[256][33];
    const int tid = threadIdx.x;
    float mx = -INFINITY;
    for (int j = tid; j < nmem + n; j += 256) mx = fmaxf(mx, j < nmem ? mk[j] : krow[j - nmem]);
    red[tid] = mx;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) { if (tid < w) red[tid] = fmaxf(red[tid], red[tid + w]); __syncthreads(); }
    mx = red[0];
    __syncthreads();
    float sm = 0.0f;
    for (int j = tid; j < nmem + n; j += 256) sm += expf((j < nmem ? mk[j] : krow[j - nmem]) - mx);
    red[tid] = sm;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) { if (tid < w) red[tid] += red[tid + w]; __syncthreads(); }
    const float inv = 1.0f / red[0];
    float s[32];
#pragma unroll
    for (int e = 0; e < 32; ++e) s[e] = 0.0f;
    for (int j = tid; j < nmem + n; j += 256) {
        const float p = expf((j < nmem ? mk[j] : krow[j - nmem]) - mx) * inv;
#pragma unroll
        for (int e = 0; e < 32; ++e)
            if (e < dh) s[e] += p * (j < nmem ? mv[(size_t)e * nmem + j] : vbase[(size_t)e * n + (j - nmem)]);
    }
#pragma unroll
    for (int e = 0; e < 32; ++e) acc[tid][e] = s[e];
    __syncthreads();
    if (tid < dh) {
        float t = 0.0f;
        for (int i = 0; i < 256; ++i) t += acc[i][tid];
        ctx[(((size_t)b * heads + h) * dh + d) * dh + tid] = t;
    }
}

// per (b, h, pixel): q softmax over d, scale, out[e] = sum_d ctx[d][e] q[d]
__global__ __launch_bounds__(256) void k_la_out(int heads, int dh, int n, float scale, const float *__restrict__ qkv,
                                                const float *__restrict__ ctx, float *__restrict__ out)
{
    const int h = blockIdx.y, b = blockIdx.z;
    const int C = heads * dh;
    __shared__ float cs[32][33];
    for (int i = threadIdx.x; i < dh * dh; i += blockDim.x) cs[i / dh][i % dh] = ctx[(((size_t)b * heads + h) * dh) * dh + i];
    __syncthreads();
    const int pix = blockIdx.x * blockDim.x + threadIdx.x;
    if (pix >= n) return;
    const float *q = qkv + ((size_t)b * 3 * C + h * dh) * n + pix;
    float qv[32];
    float mx = -INFINITY;
#pragma unroll
    for (int d = 0; d < 32; ++d) if (d < dh) { qv[d] = q[(size_t)d * n]; mx = fmaxf(mx, qv[d]); }
    float sm = 0.0f;
#pragma unroll
    for (int d = 0; d < 32; ++d) if (d < dh) { qv[d] = expf(qv[d] - mx); sm += qv[d]; }
#pragma unroll
    for (int d = 0; d < 32; ++d) if (d < dh) qv[d] = (qv[d] / sm) * scale;
    float *o = out + ((size_t)b * C + h * dh) * n + pix;
    for (int e = 0; e < dh; ++e) {
        float t = 0.0f;
#pragma unroll
        for (int d = 0; d < 32; ++d) if (d < dh) t += cs[d][e] * qv[d];
        o[(size_t)e * n] = t;
    }
}

// ---------------------------------------------------------------------------- full attention
// one workgroup per (b, h); one thread per query pixel (n <= blockDim); head width DH (32 in the U-Net)
template <int DH>
__global__ __launch_bounds__(256) void k_full_attn(int heads, int n, int nmem, const float *__restrict__ qkv,
                                                   const float *__restrict__ mem, float *__restrict__ out)
{
    constexpr int dh = DH;
    const int h = blockIdx.x, b = blockIdx.y;
    const int C = heads * dh, nk = nmem + n;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float *Ks = sm;                      // [nk][dh+1]
    float *Vs = sm + nk * (dh + 1);      // [nk][dh+1]
    const float *kb = qkv + ((size_t)b * 3 * C + C + h * dh) * n;
    const float *vb = qkv + ((size_t)b * 3 * C + 2 * C + h * dh) * n;
    for (int i = threadIdx.x; i < nk * dh; i += blockDim.x) {
        const int j = i / dh, d = i - j * dh;
        float kv, vv;
        if (j < nmem) {
            kv = mem[(((size_t)0 * heads + h) * nmem + j) * dh + d];
            vv = mem[(((size_t)1 * heads + h) * nmem + j) * dh + d];
        } else {
            kv = kb[(size_t)d * n + (j - nmem)];
            vv = vb[(size_t)d * n + (j - nmem)];
        }
        Ks[j * (dh + 1) + d] = kv;
        Vs[j * (dh + 1) + d] = vv;
    }
    __syncthreads();
    const int i = threadIdx.x;
    if (i >= n) return;
    const float *qb = qkv + ((size_t)b * 3 * C + h * dh) * n + i;
    float q[DH];
#pragma unroll
    for (int d = 0; d < dh; ++d) q[d] = qb[(size_t)d * n];
    const float scale = 1.0f / sqrtf((float)dh);
    float mx = -INFINITY;
    for (int j = 0; j < nk; ++j) {
        float s = 0.0f;
#pragma unroll
        for (int d = 0; d < dh; ++d) s += q[d] * Ks[j * (dh + 1) + d];
        mx = fmaxf(mx, s * scale);
    }
    float o[DH];
#pragma unroll
    for (int d = 0; d < dh; ++d) o[d] = 0.0f;
    float den = 0.0f;
    for (int j = 0; j < nk; ++j) {
        float s = 0.0f;
#pragma unroll
        for (int d = 0; d < dh; ++d) s += q[d] * Ks[j * (dh + 1) + d];
        const float p = expf(s * scale - mx);
        den += p;
#pragma unroll
        for (int d = 0; d < dh; ++d) o[d] += p * Vs[j * (dh + 1) + d];
    }
    float *ob = out + ((size_t)b * C + h * dh) * n + i;
#pragma unroll
    for (int d = 0; d < dh; ++d) ob[(size_t)d * n] = o[d] / den;
}

// -------------------------------------------------------------------------- RED elementwise
__global__ __launch_bounds__(256) void k_red_q_sample(int64_t n, const float *__restrict__ sa,
                                                      const float *__restrict__ s1a, const int64_t *__restrict__ t,
                                                      const float *__restrict__ x0, const float *__restrict__ eps,
                                                      float *__restrict__ xt)
{
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int b = blockIdx.y;
    if (i >= n) return;
    const int64_t tb = t[b];
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

}  // namespace

extern "C" {

int rdq_conv2d(const rdq_conv_desc *d, const float *x, const float *x2, const float *w, const float *bias,
               const float *residual, float *y, hipStream_t st)
{
    if (!d || !x || !w || !y || d->B < 1 || d->cin1 < 1 || d->cout < 1 || d->kh < 1 || d->kw < 1 || d->H < 1 ||
        d->W < 1 || (d->cin2 > 0 && !x2 && d->in_mode == RDQ_IN_PLAIN))
        return RDQ_E_INVALID;
    if (d->in_mode == RDQ_IN_UNSHUFFLE2 && (d->cin1 % 4 != 0 || d->cin2 != 0)) return RDQ_E_INVALID;
    if (d->in_mode == RDQ_IN_UPSAMPLE2 && ((d->H | d->W) & 1 || d->cin2 != 0)) return RDQ_E_INVALID;
    ConvArgs a{*d, x, x2, w, bias, residual, y};
    const int M = d->B * d->H * d->W;
    hipLaunchKernelGGL(k_conv_mfma, dim3((M + CBM - 1) / CBM, (d->cout + CBN - 1) / CBN), dim3(256), 0, st, a);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

size_t rdq_group_norm_ws_bytes(int32_t B, int32_t C, int32_t HW, int32_t G)
{
    if (B < 1 || C < 1 || HW < 1 || G < 1) return 0;
    const int64_t gsize = (int64_t)(C / G) * HW;
    const int64_t nchunk = (gsize + GN_CHUNK - 1) / GN_CHUNK;
    return (size_t)B * G * nchunk * 2 * sizeof(double);
}

int rdq_group_norm_silu(int32_t B, int32_t C, int32_t HW, int32_t G, float eps, const float *x, const float *gamma,
                        const float *beta, const float *ss, float *y, void *ws, hipStream_t st)
{
    if (B < 1 || C < 1 || HW < 1 || G < 1 || C % G || !x || !gamma || !beta || !y || !ws) return RDQ_E_INVALID;
    const int64_t gsize = (int64_t)(C / G) * HW;
    const int nchunk = (int)((gsize + GN_CHUNK - 1) / GN_CHUNK);
    double *part = (double *)ws;
    hipLaunchKernelGGL(k_gn_partial, dim3(nchunk, B * G), dim3(256), 0, st, x, gsize, nchunk, part);
    const int nb = (int)std::min<int64_t>((gsize + 255) / 256, 64);
    hipLaunchKernelGGL(k_gn_apply, dim3(nb, B * G), dim3(256), 0, st, C, HW, G, eps, nchunk, x, gamma, beta, ss, part, y);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

int rdq_rmsnorm(int32_t B, int32_t C, int32_t HW, const float *x, const float *g, const float *res, float *y,
                hipStream_t st)
{
    if (B < 1 || C < 1 || HW < 1 || !x || !g || !y) return RDQ_E_INVALID;
    hipLaunchKernelGGL(k_rmsnorm, dim3((HW + 255) / 256, B), dim3(256), 0, st, C, HW, x, g, res, y);
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

size_t rdq_linear_attention_ws_bytes(int32_t B, int32_t heads, int32_t dh)
{
    return (size_t)B * heads * dh * dh * sizeof(float);
}

int rdq_linear_attention(int32_t B, int32_t heads, int32_t dh, int32_t n, int32_t nmem, float scale, const float *qkv,
                         const float *mem_kv, float *out, void *ws, hipStream_t st)
{
    if (B < 1 || heads < 1 || dh < 1 || dh > 32 || n < 1 || nmem < 0 || !qkv || !mem_kv || !out || !ws)
        return RDQ_E_INVALID;
    float *ctx = (float *)ws;
    hipLaunchKernelGGL(k_la_context, dim3(dh, heads, B), dim3(256), 0, st, heads, dh, n, nmem, qkv, mem_kv, ctx);
    hipLaunchKernelGGL(k_la_out, dim3((n + 255) / 256, heads, B), dim3(256), 0, st, heads, dh, n, scale, qkv, ctx, out);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

int rdq_full_attention(int32_t B, int32_t heads, int32_t dh, int32_t n, int32_t nmem, const float *qkv,
                       const float *mem_kv, float *out, hipStream_t st)
{
    if (B < 1 || heads < 1 || dh != 32 || n < 1 || n > 256 || nmem < 0 || !qkv || !mem_kv || !out)
        return RDQ_E_INVALID;
    const size_t lds = (size_t)2 * (nmem + n) * (dh + 1) * sizeof(float);
    if (lds > 64 * 1024) return RDQ_E_INVALID;
    hipLaunchKernelGGL(k_full_attn<32>, dim3(heads, B), dim3(256), lds, st, heads, n, nmem, qkv, mem_kv, out);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

int rdq_red_q_sample(int32_t B, int64_t n, const float *sa, const float *s1a, const int64_t *t, const float *x0,
                     const float *eps, float *xt, hipStream_t st)
{
    if (B < 1 || n < 1 || !sa || !s1a || !t || !x0 || !eps || !xt) return RDQ_E_INVALID;
    hipLaunchKernelGGL(k_red_q_sample, dim3((unsigned)((n + 255) / 256), B), dim3(256), 0, st, n, sa, s1a, t, x0, eps, xt);
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
