// fwi.hip — MI355X (gfx950) kernels + C ABI for red-diffeq's acoustic FWI hot path.
//
// Reference behaviour (SimingShan/red-diffeq):
//   K3 rdq_fwi_coeffs      red_diffeq/solvers/pde.py:91 (replicate pad), 38-52 (get_Abc),
//                          63-71 (alpha/temp1/temp2/beta), utils/data_trans.py:13-15 (denorm)
//   K1 rdq_fwi_forward     pde.py:74-86: the whole nt-step time loop (stencil + periodic wrap + source
//                          injection + receiver sampling + history store) in ONE persistent launch when
//                          the survey fits resident (k_fwd_pt), else launches of T steps (k_fwd_tb)
//   K2 rdq_fwi_adjoint     the autograd backward of pde.py:74-86 (discrete adjoint)
//   K4 rdq_fwi_grad_finalize  chain rule back to v_norm incl. the vmin/argmin sponge term
//
// fp32 operation order follows the reference expression order exactly and the file is built
// with -ffp-contract=off, so K1 reproduces the reference seismograms bit-for-bit and K2's
// exact-order variant matches the oracle's gA accumulator bit-for-bit (tests/test_gpu_fwi.py).
//
// Data layout (HBM): padded grid Hp x Wp with row pitch ld = roundup(Wp, 64) floats (256-B
// aligned rows -> every row of a 64-wide tile is 1 or 2 full 128-B lines).
//   coeffs  [6][B][Hp][ld]       alpha, temp1, temp2, kappa, beta, v (per velocity model)
//   history [nt+2][B][ns][Hp][ld] slot j = P_{j-1}; one time step of all shots is contiguous
//   ring    [3][B][ns][Hp][ld]    rotating wavefields (no-grad forward) / adjoint lambdas
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>
#include <initializer_list>
#include <mutex>
#include <utility>

#include "red_diffeq_fwi.h"

#pragma clang fp contract(off)

namespace {

constexpr float C1X2 = -5.0f;                      // 2*c1, pde.py:66,69
constexpr float C2 = (float)(4.0 / 3.0);           // pde.py:67
constexpr float C3 = (float)(-1.0 / 12.0);         // pde.py:68

#define RDQ_CHECK(x)                                   \
    do {                                               \
        hipError_t e_ = (x);                           \
        if (e_ != hipSuccess) return -(int)e_;         \
    } while (0)
#define RDQ_TRY(x)                                     \
    do {                                               \
        const int rc_ = (x);                           \
        if (rc_ != 0) return rc_;                      \
    } while (0)


// --------------------------------------------------------------------------------------- K3
// vmin / first row-major argmin over the (unpadded) model; the padded field's first minimum
// folds back to this cell (pde.py:41, torch.min tie rule = first index).
// vmin and its first argmin per model (torch.min's tie rule, pde.py:41), in two passes: gridDim.y parts
// of each model reduce contiguous index ranges to (min, first index) partials, then one workgroup per
// model combines them (a 1.5 M-cell configs[4] model took 630 us in one workgroup).  The comparison
// (value, then index) is order-independent, so the result is the one-pass scan's bit for bit.
__device__ __forceinline__ void vstat_reduce(float &best, int64_t &bi, float *sv, int64_t *si)
{
    sv[threadIdx.x] = best;
    si[threadIdx.x] = bi;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
            const float ov = sv[threadIdx.x + w];
            const int64_t oi = si[threadIdx.x + w];
            if (ov < sv[threadIdx.x] || (ov == sv[threadIdx.x] && oi < si[threadIdx.x])) {
                sv[threadIdx.x] = ov;
                si[threadIdx.x] = oi;
            }
        }
        __syncthreads();
    }
    best = sv[0];
    bi = si[0];
}

__global__ __launch_bounds__(256) void k_vstat_part(const float *__restrict__ vn, int64_t s0, int64_t s2,
                                                    int64_t s3, int nz, int nx, int vel_mode, int chunk,
                                                    float *pv, int64_t *pi)
{
    const int b = blockIdx.x, part = blockIdx.y;
    const int n = nz * nx, i0 = part * chunk, i1 = min(n, i0 + chunk);
    float best = INFINITY;
    int64_t bi = INT64_MAX;
    // each thread's elements in increasing order, loads issued 8 at a time
    constexpr int CH = 8;
    for (int base = i0 + threadIdx.x; base < i1; base += CH * blockDim.x) {
        float t[CH];
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const int i = base + u * blockDim.x;
            const int iz = i / nx, ix = i - iz * nx;
            t[u] = i < i1 ? vn[b * s0 + iz * s2 + ix * s3] : INFINITY;
        }
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const int i = base + u * blockDim.x;
            float v = t[u];
            if (vel_mode == 0) { v = v + 1.0f; v = v / 2.0f; v = v * 3000.0f; v = v + 1500.0f; }
            if (i < i1 && v < best) { best = v; bi = i; }
        }
    }
    __shared__ float sv[256];
    __shared__ int64_t si[256];
    vstat_reduce(best, bi, sv, si);
    if (threadIdx.x == 0) {
        pv[(size_t)b * gridDim.y + part] = best;
        pi[(size_t)b * gridDim.y + part] = bi;
    }
}

__global__ __launch_bounds__(256) void k_vstat_final(const float *__restrict__ pv, const int64_t *__restrict__ pi,
                                                     int parts, float lnk, float two_a, float *vmin, int64_t *amin,
                                                     float *ks)
{
    const int b = blockIdx.x;
    float best = INFINITY;
    int64_t bi = INT64_MAX;
    for (int j = threadIdx.x; j < parts; j += blockDim.x) {
        const float v = pv[(size_t)b * parts + j];
        const int64_t i = pi[(size_t)b * parts + j];
        if (v < best || (v == best && i < bi)) { best = v; bi = i; }
    }
    __shared__ float sv[256];
    __shared__ int64_t si[256];
    vstat_reduce(best, bi, sv, si);
    if (threadIdx.x == 0) {
        vmin[b] = best;
        amin[b] = bi;
        float k = 3.0f * best; k = k * lnk; k = k / two_a;   // kappa = 3*vmin*ln(1e7)/(2a), pde.py:43
        ks[b] = k;
    }
}

// Coefficient fields at one padded-grid point (pde.py:38-52, 63-71), from the model velocity
// and the per-model sponge amplitude ks = 3*vmin*ln(1e7)/(2a).  K3 stores them for inspection and
// for K4; the time-loop kernels regenerate them in registers (bit-identical: same function), so a
// launch reads a 20 KB model instead of three 400 KB padded fields per shot.
struct CoefGen {
    const float *vmod;   // [B][nz][nx] velocity (m/s)
    const float *ks;     // [B]
    int nz, nx, nbc, Hp, Wp;
    float dt, dx, a;
};

struct Coef { float v, al, t1, t2, kp; };

__device__ __forceinline__ Coef gen_coef(const CoefGen &c, int b, int z, int x)
{
    const int iz = min(max(z - c.nbc, 0), c.nz - 1);
    const int ix = min(max(x - c.nbc, 0), c.nx - 1);
    Coef o;
    o.v = c.vmod[((size_t)b * c.nz + iz) * c.nx + ix];
    const int nbc = c.nbc;
    int pi = -1;                                   // rows first, then columns overwrite (corners)
    if (z < nbc) pi = nbc - 1 - z;
    if (z >= c.Hp - nbc) pi = z - (c.Hp - nbc);
    if (x < nbc) pi = nbc - 1 - x;
    if (x >= c.Wp - nbc) pi = x - (c.Wp - nbc);
    float dmp = 0.0f;
    if (pi >= 0) { float d = (float)pi * c.dx; d = d / c.a; d = d * d; dmp = c.ks[b] * d; }
    float al = o.v * c.dt; al = al / c.dx; al = al * al;                   // pde.py:63
    o.al = al;
    o.kp = dmp * c.dt;                                                      // pde.py:65
    float t1 = C1X2 * al; t1 = t1 + 2.0f; t1 = t1 - o.kp;                   // pde.py:69
    o.t1 = t1;
    o.t2 = 1.0f - o.kp;                                                     // pde.py:70
    return o;
}

__device__ __forceinline__ float beta_of(float v, float dt) { float bt = v * dt; return bt * bt; }  // pde.py:71

struct CoefArgs {
    const float *vn;
    int64_t s0, s2, s3;
    int vel_mode, ld;
    CoefGen cg;
    float *vmod_out;
    float *coeffs;
    size_t cstride;  // B*Hp*ld
};

__global__ __launch_bounds__(256) void k_coeffs(CoefArgs p)
{
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int z = blockIdx.y;
    const int b = blockIdx.z;
    const CoefGen &c = p.cg;
    if (x >= p.ld) return;
    const size_t i = ((size_t)b * c.Hp + z) * p.ld + x;
    if (x >= c.Wp) {
        for (int f = 0; f < 6; ++f) p.coeffs[f * p.cstride + i] = 0.0f;
        return;
    }
    const int iz = z - c.nbc, ix = x - c.nbc;
    if (iz >= 0 && iz < c.nz && ix >= 0 && ix < c.nx) {   // the model itself (unpadded)
        float v = p.vn[b * p.s0 + iz * p.s2 + ix * p.s3];
        if (p.vel_mode == 0) { v = v + 1.0f; v = v / 2.0f; v = v * 3000.0f; v = v + 1500.0f; }  // data_trans.py:15
        p.vmod_out[((size_t)b * c.nz + iz) * c.nx + ix] = v;
    }
}

__global__ __launch_bounds__(256) void k_coeff_fields(CoefArgs p)
{
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int z = blockIdx.y;
    const int b = blockIdx.z;
    const CoefGen &c = p.cg;
    if (x >= c.Wp) return;
    const size_t i = ((size_t)b * c.Hp + z) * p.ld + x;
    const Coef o = gen_coef(c, b, z, x);
    p.coeffs[i] = o.al;
    p.coeffs[p.cstride + i] = o.t1;
    p.coeffs[2 * p.cstride + i] = o.t2;
    p.coeffs[3 * p.cstride + i] = o.kp;
    p.coeffs[4 * p.cstride + i] = beta_of(o.v, c.dt);
    p.coeffs[5 * p.cstride + i] = o.v;
}

// buffer addressing: scalar base + 32-bit lane offset; an offset past the range is dropped (no
// memory access; loads return 0)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void *base, int bytes = 0x7fffffff)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, bytes, 0x00020000);
}
constexpr int OOB = (int)0x80000000u;               // buffer offset beyond every range: store dropped
// buffer cache policy "nt" (non-temporal, streaming): the history stream is written once and read
// once, GBs apart; without the hint it churns the L2 that carries the persistent kernels' hand-offs
// (their first sweep pass: 306 -> 220 us per forward launch, 299 -> 214 us per adjoint launch)
constexpr int CP_NT = 2;
__device__ __forceinline__ float bload(__amdgpu_buffer_rsrc_t r, int voff, int soff)
{
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}
// --------------------------------------------------------------------------------------- K1/K2
// Temporal blocking on a register-resident region (the MI355X design of the time loop).
//
// A workgroup of NW waves owns a region of 64 columns (one per lane) x NW*R rows (R consecutive
// rows per wave, held in VGPRs) of one (model, shot) slice, and advances it T time steps per
// launch.  Halo H = 2T on every side: after t steps the outermost 2t rows/columns are stale, the
// interior (64-2H) x (NW*R-2H) stays exact and is the only part that is stored.  Per step:
//   - vertical taps: the wave's own registers; the two rows above/below its slab come from the
//     neighbouring waves through a 2 KB LDS exchange (double-buffered: one barrier per step);
//   - horizontal taps: DPP wave shifts (v_mov_b32_dpp wave_shr:1 / wave_shl:1) — no LDS traffic;
//   - periodic wrap (torch.roll, pde.py:79) is in the region->grid map (global index mod Hp/Wp),
//     so a tile at the domain edge simply loads wrapped rows/columns.
// T steps per launch divide the launch count (the latency floor of the per-step design) by T and
// cut the wavefield re-reads to two levels per launch; the extra arithmetic is the halo.
constexpr int TB_NW = 8;                 // waves per workgroup
constexpr int TB_R = 8;                  // rows per wave
constexpr int TB_RH = TB_NW * TB_R;      // region rows
constexpr int TB_MAXT = 4;
constexpr int TW_FWD_MAXT = 6;          // deepest wide chunked forward (k_fwd_tw instantiations 1 .. 6)
constexpr int FWD_W_MAX = TW_FWD_MAXT > TB_MAXT ? TW_FWD_MAXT : TB_MAXT;   // wavelet samples per chunked forward launch

__device__ __forceinline__ float dpp_shr1(float v)   // lane i <- lane i-1 (x-1); lane 0 reads 0
{
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float dpp_shl1(float v)   // lane i <- lane i+1 (x+1); lane 63 reads 0
{
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x130, 0xf, 0xf, true));
}

struct TBGeo {
    int B, ns, Hp, Wp, ld, isz, igz, ng, nrec, st;
    int s_off, ns_grp;                   // chunked launch: shots [s_off, s_off + ns_grp) of all B models
    int sl_off, nsl;                     // persistent launch: flat slices [sl_off, sl_off + nsl), slice = b * ns + s
    int tiles_x, ntiles;                 // tile grid of this launch's blocking depth
    size_t cstride, slice, level;        // level = B*ns*slice (one time level of all slices)
    const int *isx, *rcv_start, *rcv_list;
    const int *rlane;                    // [Wp] adjoint residual index of a column (-1: no receiver)
    int dstride;                         // residual row stride: ng, or ncolr after the fold
};

struct FwdTBArgs {
    TBGeo g;
    CoefGen cg;                          // model + sponge amplitude (GEN variant)
    const float *coeffs;                 // K3 fields: alpha, temp1, temp2 at 0, 1, 2 x cstride
    const float *in_prev, *in_cur;       // P_{n-1}, P_n   (each [B][ns][Hp][ld])
    float *hist;                         // history base (slot j = P_{j-1}) or nullptr
    float *out_prev, *out_cur;           // ring path: P_{n+T-1}, P_{n+T}
    float *seis;
    int n0, nsteps;
    int spw, ns_sh;                      // wide kernels: shots per workgroup, shots of the launch's chain
    float w[FWD_W_MAX];                  // wavelet samples w[n0 .. n0+nsteps-1]
};

// exchange two boundary rows each way between the NW waves of the workgroup
struct Halo4 { float u2, u1, d1, d2; };

__device__ __forceinline__ Halo4 exchange(float (*xch)[TB_NW][4][64], int buf, int w, int lane,
                                          float top0, float top1, float bot1, float bot0)
{
    xch[buf][w][0][lane] = top0;      // row 0
    xch[buf][w][1][lane] = top1;      // row 1
    xch[buf][w][2][lane] = bot1;      // row R-2
    xch[buf][w][3][lane] = bot0;      // row R-1
    __syncthreads();
    Halo4 h;
    const int wu = w > 0 ? w - 1 : 0, wd = w < TB_NW - 1 ? w + 1 : TB_NW - 1;
    h.u2 = xch[buf][wu][2][lane];     // row -2 (garbage for w == 0: outside the region)
    h.u1 = xch[buf][wu][3][lane];     // row -1
    h.d1 = xch[buf][wd][0][lane];     // row R
    h.d2 = xch[buf][wd][1][lane];     // row R+1
    return h;
}

template <int NW>
__device__ __forceinline__ Halo4 exchange_nw(float (*xch)[NW][4][64], int buf, int w, int lane, float top0,
                                             float top1, float bot1, float bot0)
{
    xch[buf][w][0][lane] = top0;
    xch[buf][w][1][lane] = top1;
    xch[buf][w][2][lane] = bot1;
    xch[buf][w][3][lane] = bot0;
    __syncthreads();
    Halo4 h;
    const int wu = w > 0 ? w - 1 : 0, wd = w < NW - 1 ? w + 1 : NW - 1;
    h.u2 = xch[buf][wu][2][lane];
    h.u1 = xch[buf][wu][3][lane];
    h.d1 = xch[buf][wd][0][lane];
    h.d2 = xch[buf][wd][1][lane];
    return h;
}

// ---- Barrier-free wave-to-wave exchange of the persistent forward and adjoint.  Each step a wave
// needs two rows above and below its own from its neighbour waves; instead of a workgroup barrier per
// step, each wave waits only for the two waves it reads from, and publishes its boundary rows as soon
// as they are computed (its interior rows follow), so the neighbours' rows are normally there at the
// first read.  History of the form (configs[1], profiles/r3/barrier_free_ab.txt, profiles/r6/
// fwd_xf_ab.txt, mailbox_ab.txt): 16-byte tagged slots {row, tag, row, tag} (round 3: forward 1.364 ->
// 1.31 ms); a per-lane flag word after the rows, which drops the 8 register moves that built the
// tagged slots and the 6 compares that checked them (1.208 -> 1.111 ms with the trims of the same
// change; every instruction a wave issues sits on the step's path: profiles/r6/issue_pad_ab.txt); the
// mailbox below (same speed for the forward, adjoint 1.560 -> 1.548 ms: it needs fewer VGPRs, which
// the 128-VGPR adjoint has none of).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 fma2(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
constexpr unsigned XQ_NONE = 0xFFFFFFFFu;                 // flag of a never-written inbox
// Wave priorities of the barrier-free persistent kernels (s_setprio; the SIMD's arbiter issues the
// higher-priority wave first).  A wave polling its LDS inbox (xm_wait) or the hand-off
// granules (PT_SWEEP) drops to WAIT, so its spin loop does not take issue cycles from the waves still
// computing; a wave that got its neighbours' rows runs its two boundary row pairs (what the neighbours
// wait for next) at EDGE, then its interior pairs at BODY.  Configs[1] forward, interleaved x3
// (profiles/r6/wave_priority_ab.txt): 1.342 -> 1.262 ms with the LDS spin alone at WAIT, 1.225 with the
// sweep too, 1.212 with the edge / body split; 1.362 -> 1.204 ms against no priorities in a second run,
// 1.194 with the post-sweep priority at EDGE (the default) and 1.217 with BODY = 2.  (With a barrier
// per step the adjoint gained nothing, 1.638 -> 1.646 ms with the sweep at WAIT; its barrier-free form,
// ADJR_STEP_NB, uses the same exchange and priorities: 1.646 -> 1.577 ms.)
constexpr int PT_PRIO_WAIT = 0, PT_PRIO_BODY = 1, PT_PRIO_SWEPT = 3, PT_PRIO_EDGE = 3;
// ---- Mailbox exchange (xm_*): each wave owns an inbox per buffer, {rows -1, R, -2, R+1} as 16 bytes
// (halo pairs E1 = {-1, R}, E2 = {-2, R+1}: one ds_read_b128 straight into them) and a flag pair
// {from above, from below}.  A wave writes its rows R-1, R-2 into the lower wave's inbox and its rows
// 0, 1 into the upper wave's (ds_write2_b32 straight from its row-pair registers), each followed by
// its flag there (the step's tag); waves 0 / NW-1 fill their own inbox's missing half (rows outside
// the region: any value, the halo absorbs it).  A wave's LDS instructions execute in order, so a
// reader that reads its flags before its rows and finds both tags reads rows written before them;
// buffer reuse is safe without a barrier (a wave writes step n+1's rows only after it read its step-n inbox,
// whose writers wrote it after reading their step n-1 inboxes).  Per step and wave: 4 writes, 2 reads
// and 2 compares, no register moves on either side.
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) f32x4 lds_f32x4;
typedef __attribute__((address_space(3))) u32x2 lds_u32x2;
typedef __attribute__((address_space(3))) float lds_float;
typedef __attribute__((address_space(3))) unsigned lds_uint;
template <int NW> struct XmBox { f32x4 rows[2][NW][64]; u32x4 flags[2][NW][64]; };   // [buffer][wave][lane]
template <int NW>
__device__ __forceinline__ void xm_init(XmBox<NW> &m, int w, int lane)
{
    const u32x4 z = {XQ_NONE, XQ_NONE, 0u, 0u};
    m.flags[0][w][lane] = z;
    m.flags[1][w][lane] = z;
}
// p0 = rows {0, R-1}, p1 = rows {1, R-2} (mirrored pairs 0, 1)
template <int NW>
__device__ __forceinline__ void xm_put(XmBox<NW> &m, int buf, int w, int lane, unsigned tag, f32x2 p0, f32x2 p1)
{
    constexpr int FLAGS = NW * 64 * 4 * 2;                // flags[buf] - rows[buf] in floats (same layout)
    lds_float *dn = (lds_float *)&m.rows[buf][w < NW - 1 ? w + 1 : w][lane] + (w < NW - 1 ? 0 : 1);
    lds_float *up = (lds_float *)&m.rows[buf][w > 0 ? w - 1 : w][lane] + (w > 0 ? 1 : 0);
    dn[0] = p0.y; dn[2] = p1.y;                           // the lower wave's rows -1, -2
    up[0] = p0.x; up[2] = p1.x;                           // the upper wave's rows R, R+1
    asm volatile("" ::: "memory");                        // rows before flags (program order = LDS order)
    ((lds_uint *)dn)[FLAGS] = tag;
    ((lds_uint *)up)[FLAGS] = tag;
}
template <int NW>
__device__ __forceinline__ void xm_load(XmBox<NW> &m, int buf, int w, int lane, u32x2 &f, f32x2 &E1, f32x2 &E2)
{
    asm volatile("" ::: "memory");
    f = *(const lds_u32x2 *)&m.flags[buf][w][lane];
    asm volatile("" ::: "memory");                        // flags before rows
    const f32x4 e = *(const lds_f32x4 *)&m.rows[buf][w][lane];
    E1 = f32x2{e.x, e.y};
    E2 = f32x2{e.z, e.w};
}
__device__ __forceinline__ bool xm_ready(u32x2 f, unsigned tag)
{
    return (__builtin_amdgcn_ballot_w64(f.x == tag) & __builtin_amdgcn_ballot_w64(f.y == tag)) == ~0ull;
}
template <int NW>
__device__ __forceinline__ void xm_wait(XmBox<NW> &m, int buf, int w, int lane, unsigned tag, u32x2 f, f32x2 &E1,
                                        f32x2 &E2, unsigned *status, bool &live)
{
    if (!xm_ready(f, tag)) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        __builtin_amdgcn_s_setprio(PT_PRIO_WAIT);        // (see PT_PRIO_*)
        for (unsigned it = 1;; ++it) {
            xm_load<NW>(m, buf, w, lane, f, E1, E2);
            if (xm_ready(f, tag)) break;
            if (!live) break;
            if ((it & 255u) == 0 && __builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {   // 1 s
                __hip_atomic_store(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                live = false;
                break;
            }
        }
    }
    __builtin_amdgcn_s_setprio(PT_PRIO_EDGE);
}


// the same for two fields with ONE barrier (adjoint: A*L_{k+1} and the history P_{k-1})
__device__ __forceinline__ void exchange2(float (*xa)[TB_NW][4][64], float (*xb)[TB_NW][4][64], int buf, int w,
                                          int lane, const float (&fa)[4], const float (&fb)[4], Halo4 &ha,
                                          Halo4 &hb)
{
#pragma unroll
    for (int i = 0; i < 4; ++i) { xa[buf][w][i][lane] = fa[i]; xb[buf][w][i][lane] = fb[i]; }
    __syncthreads();
    const int wu = w > 0 ? w - 1 : 0, wd = w < TB_NW - 1 ? w + 1 : TB_NW - 1;
    ha.u2 = xa[buf][wu][2][lane]; ha.u1 = xa[buf][wu][3][lane]; ha.d1 = xa[buf][wd][0][lane]; ha.d2 = xa[buf][wd][1][lane];
    hb.u2 = xb[buf][wu][2][lane]; hb.u1 = xb[buf][wu][3][lane]; hb.d1 = xb[buf][wd][0][lane]; hb.d2 = xb[buf][wd][1][lane];
}

// vertical neighbour rows of row r from the slab + halo rows
#define TB_VERT(ARR, r, H4, m2, m1, p1, p2)                                   \
    const float m2 = (r) >= 2 ? ARR[(r) - 2] : ((r) == 1 ? H4.u1 : H4.u2);    \
    const float m1 = (r) >= 1 ? ARR[(r) - 1] : H4.u1;                        \
    const float p1 = (r) + 1 < TB_R ? ARR[(r) + 1] : H4.d1;                  \
    const float p2 = (r) + 2 < TB_R ? ARR[(r) + 2] : ((r) + 2 == TB_R ? H4.d1 : H4.d2);

// XCD-aware block -> (tile, shot) map.  Blocks are dealt round-robin over the 8 XCDs (block b
// and b+8 share an L2); every shot of one tile gets the same (block mod 8), so the per-model
// coefficient rows a tile reads are fetched once per XCD and re-read from that L2 by the other
// shots of the group.  A placement guess only changes speed, never results.
struct TileId { int tx, ty, tile, sl; bool valid; };

__host__ __device__ __forceinline__ TileId decode_tile(int L, int tiles_x, int ntiles, int nsg)
{
    TileId t;
    t.tile = (L / (8 * nsg)) * 8 + (L & 7);
    t.sl = (L >> 3) % nsg;
    t.valid = t.tile < ntiles;
    t.ty = t.tile / tiles_x;
    t.tx = t.tile - t.ty * tiles_x;
    return t;
}

// record index of time step n under sample_temporal st (-1: not a recorded step); st == 1, the
// reference default, needs no integer division
__device__ __forceinline__ int rec_index(int n, int st)
{
    if (st == 1) return n;
    return (n % st) == 0 ? n / st : -1;
}

// cheap wrap for |v| < a few n (general v handled by the loops)
__device__ __forceinline__ int wrapn(int v, int n)
{
    while (v < 0) v += n;
    while (v >= n) v -= n;
    return v;
}

template <int T, bool GEN>
__global__ __launch_bounds__(64 * TB_NW) void k_fwd_tb(FwdTBArgs a)
{
    constexpr int H = 2 * T, IW = 64 - 2 * H, IH = TB_RH - 2 * H;
    __shared__ float xch[2][TB_NW][4][64];
    const TBGeo &g = a.g;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform
    const TileId ti = decode_tile(blockIdx.x, g.tiles_x, g.ntiles, g.B * g.ns_grp);
    if (!ti.valid) return;                                            // whole workgroup: uniform
    const int b = ti.sl / g.ns_grp, s = g.s_off + (ti.sl - b * g.ns_grp), bs = b * g.ns + s;
    const int ux = ti.tx * IW - H + lane;                             // unwrapped column
    const int gx = wrapn(ux, g.Wp);
    const bool xin = lane >= H && lane < 64 - H && ux < g.Wp;
    const int uz0 = ti.ty * IH - H + w * TB_R;                        // unwrapped row of r = 0
    const size_t so = (size_t)bs * g.slice;
    const float *AL = a.coeffs + (size_t)b * g.slice;
    const float *T1p = AL + g.cstride, *T2p = AL + 2 * g.cstride;
    const int isx = g.isx[s];
    float A[TB_R], C1[TB_R], C2v[TB_R], P0[TB_R], P1[TB_R];
    int rofs[TB_R];                 // wave-uniform row offsets gz*ld
    unsigned rin = 0;               // wave-uniform: row is interior and inside the domain
    int srow = -1, rrow = -1;       // wave-uniform: row holding the source / the receivers
#pragma unroll
    for (int r = 0; r < TB_R; ++r) {
        const int uz = uz0 + r, gz = wrapn(uz, g.Hp);
        rofs[r] = gz * g.ld;
        const int o = rofs[r] + gx;
        if constexpr (GEN) {   // regenerate from the 20 KB model (L1-resident) instead of 3 fields
            const Coef cf = gen_coef(a.cg, b, gz, gx);
            A[r] = cf.al; C1[r] = cf.t1; C2v[r] = cf.t2;
        } else {
            A[r] = AL[o]; C1[r] = T1p[o]; C2v[r] = T2p[o];
        }
        P0[r] = a.in_prev[so + o];
        P1[r] = a.in_cur[so + o];
        const int rr = w * TB_R + r;
        if (rr >= H && rr < TB_RH - H && uz < g.Hp) rin |= 1u << r;
        if (gz == g.isz) srow = r;          // (a region row maps to one grid row: one hit per wave
        if (gz == g.igz) rrow = r;          //  unless the region wraps a tiny domain -> see below)
    }
    // tiny domains (region taller than Hp) can hold the source row twice: keep every hit
    unsigned smask = 0;
#pragma unroll
    for (int r = 0; r < TB_R; ++r) if (wrapn(uz0 + r, g.Hp) == g.isz) smask |= 1u << r;
    const bool scol = gx == isx;
    const float bsrc = (smask != 0) ? a.coeffs[4 * g.cstride + (size_t)b * g.slice + (size_t)g.isz * g.ld + isx] : 0.0f;
    const int rs = (rrow >= 0) ? g.rcv_start[gx] : 0, re = (rrow >= 0) ? g.rcv_start[gx + 1] : 0;
    // this lane's (usually only) receiver, read once: a per-step index load would put an L2 round
    // trip in front of every step's seismogram store
    const int rcv0 = rs < re ? g.rcv_list[rs] : -1;
    const bool rmulti = __any(re - rs > 1);               // wave-uniform: a column with several receivers
    (void)srow;
#pragma unroll
    for (int t = 0; t < T; ++t) {
        if (t >= a.nsteps) break;
        float *cur = (t & 1) ? P0 : P1;     // P_{n+t}
        float *prv = (t & 1) ? P1 : P0;     // P_{n+t-1}  -> overwritten with P_{n+t+1}
        const Halo4 h4 = exchange(xch, t & 1, w, lane, cur[0], cur[1], cur[TB_R - 2], cur[TB_R - 1]);
#pragma unroll
        for (int r = 0; r < TB_R; ++r) {
            TB_VERT(cur, r, h4, zm2, zm1, zp1, zp2)
            const float c = cur[r];
            const float xl1 = dpp_shr1(c), xr1 = dpp_shl1(c);
            const float xl2 = dpp_shr1(xl1), xr2 = dpp_shl1(xr1);
            // pde.py:79, reference evaluation order
            float s1 = zm1 + zp1; s1 = s1 + xl1; s1 = s1 + xr1;
            float s2 = zm2 + zp2; s2 = s2 + xl2; s2 = s2 + xr2;
            float lap = C2 * s1; const float l2 = C3 * s2; lap = lap + l2;
            float a1 = C1[r] * c; const float a2 = C2v[r] * prv[r]; a1 = a1 - a2;
            const float a3 = A[r] * lap;
            prv[r] = a1 + a3;
        }
        if (smask) {                                                   // pde.py:80-81
#pragma unroll
            for (int r = 0; r < TB_R; ++r)
                if ((smask & (1u << r)) && scol) { const float add = bsrc * a.w[t]; prv[r] = prv[r] + add; }
        }
        const int n = a.n0 + t;
        if (a.hist && xin) {
            float *HS = a.hist + (size_t)(n + 2) * g.level + so + gx;
#pragma unroll
            for (int r = 0; r < TB_R; ++r)
                if (rin & (1u << r)) __builtin_nontemporal_store(prv[r], &HS[rofs[r]]);   // streaming
        }
        if (rrow >= 0 && (rin & (1u << rrow)) && xin && (n % g.st) == 0) {   // pde.py:82-83
            float val = 0.0f;
#pragma unroll
            for (int r = 0; r < TB_R; ++r) if (r == rrow) val = prv[r];
            float *SK = a.seis + ((size_t)bs * g.nrec + n / g.st) * g.ng;
            if (rcv0 >= 0) SK[rcv0] = val;
            if (rmulti)
                for (int j = rs + 1; j < re; ++j) SK[g.rcv_list[j]] = val;
        }
    }
    if (a.out_cur && xin) {   // ring path: keep the last two levels
        const bool odd = (a.nsteps & 1) != 0;   // after nsteps steps the newest level is in P0 if odd
#pragma unroll
        for (int r = 0; r < TB_R; ++r)
            if (rin & (1u << r)) {
                const size_t o = so + rofs[r] + gx;
                a.out_cur[o] = odd ? P0[r] : P1[r];
                a.out_prev[o] = odd ? P1[r] : P0[r];
            }
    }
}

constexpr int TW_ADJ_MAXT = 6;          // deepest wide chunked adjoint (k_adj_tw instantiations 1 .. 6)
constexpr int ADJ_W_MAX = TW_ADJ_MAXT > TB_MAXT ? TW_ADJ_MAXT : TB_MAXT;   // wavelet samples per chunked adjoint launch
struct AdjTBArgs {
    TBGeo g;
    CoefGen cg;                          // model + sponge amplitude (wide kernels regenerate alpha / kappa)
    const float *coeffs;                 // K3 fields: alpha, temp1, temp2, kappa at 0..3 x cstride
    const float *in_l1, *in_l2;          // L_{k0+1}, L_{k0+2}
    float *out_l1, *out_l2;              // L_{k0-nsteps+1}, L_{k0-nsteps+2}
    const float *hist;                   // slot k = P_{k-1}
    const float *dseis;
    float *gA;                           // [B][ns][Hp][ld]
    double *gk_part;                     // [B*ns][nblk]
    float *gbeta;                        // [B*ns]
    int k0, nsteps, nblk;
    int spw, ns_sh;                      // wide kernels: shots per workgroup, shots of the launch's chain
    float w[ADJ_W_MAX];                  // w[k0-1-t], t < nsteps (narrow: <= TB_MAXT, wide: <= TW_ADJ_MAXT steps)
};

// Adjoint with the same register-region blocking, walking k = k0, k0-1, ...:
//   L_k = T1 L_{k+1} - T2 L_{k+2} + (c2 N1(A L_{k+1}) + c3 N2(A L_{k+1})) [+ R^T dseis[k-1]]
// and, on the interior only, the per-shot accumulators (loaded once, stored once per launch):
//   gA_s += L_k (2c1 P_{k-1} + c2 S1(P_{k-1}) + c3 S2(P_{k-1})),  gk += (K P_{k-1})(L_{k+1} - L_k),
//   gbeta[s] += L_k(src) w[k-1].
template <int T>
__global__ __launch_bounds__(64 * TB_NW, 4) void k_adj_tb(AdjTBArgs a)
{
    constexpr int H = 2 * T, IW = 64 - 2 * H, IH = TB_RH - 2 * H;
    __shared__ float xch[2][TB_NW][4][64];
    __shared__ float pxc[2][TB_NW][4][64];
    __shared__ double red[64 * TB_NW];
    const TBGeo &g = a.g;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const TileId ti = decode_tile(blockIdx.x, g.tiles_x, g.ntiles, g.B * g.ns_grp);
    if (!ti.valid) return;                                            // whole workgroup: uniform
    const int b = ti.sl / g.ns_grp, s = g.s_off + (ti.sl - b * g.ns_grp), bs = b * g.ns + s;
    const int ux = ti.tx * IW - H + lane;
    const int gx = wrapn(ux, g.Wp);
    const bool xin = lane >= H && lane < 64 - H && ux < g.Wp;
    const int uz0 = ti.ty * IH - H + w * TB_R;
    const size_t so = (size_t)bs * g.slice;
    const float *AL = a.coeffs + (size_t)b * g.slice;
    const float *KAp = AL + 3 * g.cstride;
    const int isx = g.isx[s];
    float A[TB_R], L0[TB_R], L1[TB_R];   // temp1/temp2 are re-derived from A and K (bit-identical)
    float gal[TB_R], kal[TB_R];          // gA_s accumulators and the sponge coefficient K, in registers
    int rofs[TB_R];
    unsigned rin = 0, pmask = 0, smask = 0, rmask = 0;   // wave-uniform row masks
#pragma unroll
    for (int r = 0; r < TB_R; ++r) {
        const int uz = uz0 + r, gz = wrapn(uz, g.Hp);
        rofs[r] = gz * g.ld;
        const int o = rofs[r] + gx;
        A[r] = AL[o];                // (regenerating alpha / K from the model, as the forward does,
        kal[r] = KAp[o];             //  measured 5% slower here: the loads are cheaper than the math)
        L1[r] = a.in_l1[so + o];     // L_{k+1}
        L0[r] = a.in_l2[so + o];     // L_{k+2}
        const int rr = w * TB_R + r;
        if (rr >= H && rr < TB_RH - H && uz < g.Hp) rin |= 1u << r;
        if (rr >= H - 2 && rr < TB_RH - H + 2) pmask |= 1u << r;
        if (gz == g.isz) smask |= 1u << r;
        if (gz == g.igz) rmask |= 1u << r;
        gal[r] = ((rin & (1u << r)) && xin) ? a.gA[so + o] : 0.0f;
    }
    const bool scol = gx == isx;
    // residual of this lane's column: one receiver's dseis, or several receivers' folded sum
    const int rcv0 = rmask ? g.rlane[gx] : -1;
    const float *DSb = a.dseis + (size_t)bs * g.nrec * g.dstride;
    // gbeta of this shot accumulates in a register over the launch's steps (same order as a
    // per-step read-modify-write of a.gbeta[bs]), stored once at the end
    const bool gbl = (smask & rin) && scol && xin;       // the source cell is this lane's own cell
    float gbacc = gbl ? a.gbeta[bs] : 0.0f;
    double ksum = 0.0;
    // history P_{k-1} on the rows whose stencil the interior needs: HBM stream, prefetched one
    // step ahead so its latency hides under the previous step
    // Buffer loads with an out-of-range offset outside pmask (no memory access, returns 0): no
    // select on the loaded value, so the compiler need not wait for each load in turn.
    float Pn[TB_R];
    int pofs[TB_R];
#pragma unroll
    for (int r = 0; r < TB_R; ++r) pofs[r] = (pmask & (1u << r)) ? (rofs[r] + gx) * 4 : OOB;
    const int slice_bytes = (int)(g.slice * 4);
    {
        const __amdgpu_buffer_rsrc_t HR = rsrc_of(a.hist + (size_t)a.k0 * g.level + so, slice_bytes);
#pragma unroll
        for (int r = 0; r < TB_R; ++r) Pn[r] = bload(HR, pofs[r], 0);   // (not nt: vertically adjacent
    }                                                                          //  tiles re-read halo rows from L2)
#pragma unroll
    for (int t = 0; t < T; ++t) {
        if (t >= a.nsteps) break;
        const int k = a.k0 - t;
        float *cur = (t & 1) ? L0 : L1;     // L_{k+1}
        float *prv = (t & 1) ? L1 : L0;     // L_{k+2} -> overwritten with L_k
        float P[TB_R];
#pragma unroll
        for (int r = 0; r < TB_R; ++r) P[r] = Pn[r];
        if (t + 1 < a.nsteps) {
            const __amdgpu_buffer_rsrc_t HR = rsrc_of(a.hist + (size_t)(k - 1) * g.level + so, slice_bytes);
#pragma unroll
            for (int r = 0; r < TB_R; ++r) Pn[r] = bload(HR, pofs[r], 0);
        }
        // this step's receiver residual, loaded before the stencil so its latency hides under it
        const bool rstep = rmask && ((k - 1) % g.st) == 0;   // wave-uniform
        const float dsv = (rstep && rcv0 >= 0) ? DSb[(size_t)((k - 1) / g.st) * g.dstride + rcv0] : -0.0f;
        float q[TB_R];
#pragma unroll
        for (int r = 0; r < TB_R; ++r) q[r] = A[r] * cur[r];
        Halo4 h4, hp;
        const float qe[4] = {q[0], q[1], q[TB_R - 2], q[TB_R - 1]};
        const float pe[4] = {P[0], P[1], P[TB_R - 2], P[TB_R - 1]};
        exchange2(xch, pxc, t & 1, w, lane, qe, pe, h4, hp);
#pragma unroll
        for (int r = 0; r < TB_R; ++r) {
            TB_VERT(q, r, h4, qm2, qm1, qp1, qp2)
            const float qc = q[r];
            const float xl1 = dpp_shr1(qc), xr1 = dpp_shl1(qc);
            const float xl2 = dpp_shr1(xl1), xr2 = dpp_shl1(xr1);
            float n1 = qm1 + qp1; n1 = n1 + xl1; n1 = n1 + xr1;
            float n2 = qm2 + qp2; n2 = n2 + xl2; n2 = n2 + xr2;
            float nb = C2 * n1; const float nb2 = C3 * n2; nb = nb + nb2;
            const float kp = kal[r];
            float t1 = C1X2 * A[r]; t1 = t1 + 2.0f; t1 = t1 - kp;     // pde.py:69
            const float t2 = 1.0f - kp;                               // pde.py:70
            float l = t1 * cur[r]; const float l2 = t2 * prv[r]; l = l - l2; l = l + nb;
            prv[r] = l;
        }
        if (rstep) {                            // adjoint of the receiver sampling
#pragma unroll
            for (int r = 0; r < TB_R; ++r)
                if (rmask & (1u << r)) prv[r] = prv[r] + dsv;     // -0 on lanes without a receiver
        }
        // gradient accumulators on the interior (P halo rows came with the same exchange)
#pragma unroll
        for (int r = 0; r < TB_R; ++r) {
            TB_VERT(P, r, hp, pm2, pm1, pp1, pp2)
            const float pc = P[r];
            const float xl1 = dpp_shr1(pc), xr1 = dpp_shl1(pc);
            const float xl2 = dpp_shr1(xl1), xr2 = dpp_shl1(xr1);
            if ((rin & (1u << r)) && xin) {
                float s1 = pm1 + pp1; s1 = s1 + xl1; s1 = s1 + xr1;
                float s2 = pm2 + pp2; s2 = s2 + xl2; s2 = s2 + xr2;
                float lap = C2 * s1; const float lq = C3 * s2; lap = lap + lq;
                float d = C1X2 * pc; d = d + lap;
                const float l = prv[r];
                const float c = l * d;
                float &ga = gal[r];
                ga = ga + c;
                float kk = kal[r] * pc; const float dl = cur[r] - l; kk = kk * dl;  // fp32 term,
                ksum += (double)kk;                                                             // fp64 sum
                if ((smask & (1u << r)) && scol) { const float gb = l * a.w[t]; gbacc = gbacc + gb; }
            }
        }
    }
    if (xin) {
        const bool odd = (a.nsteps & 1) != 0;   // newest level (L_{k0-nsteps+1}) is in L0 if odd
#pragma unroll
        for (int r = 0; r < TB_R; ++r)
            if (rin & (1u << r)) {
                const size_t o = so + rofs[r] + gx;
                a.out_l1[o] = odd ? L0[r] : L1[r];
                a.out_l2[o] = odd ? L1[r] : L0[r];
                a.gA[o] = gal[r];
            }
    }
    if (gbl) a.gbeta[bs] = gbacc;
    // deterministic workgroup reduction of the sponge-coefficient partial sum
    const int tid = threadIdx.x;
    red[tid] = ksum;
    __syncthreads();
    for (int w2 = 32 * TB_NW; w2 > 0; w2 >>= 1) {
        if (tid < w2) red[tid] += red[tid + w2];
        __syncthreads();
    }
    if (tid == 0) a.gk_part[(size_t)bs * a.nblk + ti.tile] += red[0];
}

// --------------------------------------------------------------------------------------- K1/K2
// Chunked kernels on WIDE regions (configs[4]-size grids; the default chunked layout).  A region is
// 128 columns x NW*R rows: every lane holds TWO adjacent columns {2l, 2l+1} of R rows as one f32x2
// per row, so every add / mul of the stencil is one packed v_pk_*_f32 for two cells, and the
// horizontal taps of a column pair need four DPP lane shifts (x-1 of column 2l is lane l-1's .y, x-2
// its .x; x+1 of column 2l+1 is lane l+1's .x, x+2 its .y) instead of four per cell.  The region's
// halo H = 2T is then 16 of 128 columns instead of 16 of 64: a tile re-reads (128 x RH) / (112 x IH)
// of what it stores instead of (64 x 64) / (48 x 48), and its 512-B rows span 4-5 128-B lines per
// 112 owned columns instead of 3 per 48 (profiles/r3: the 64-column adjoint moved 1.34x its
// algorithmic bytes at configs[4]).  Same per-cell operations in the same order as k_fwd_tb /
// k_adj_tb (bit-exact with them and with the oracle).  PAIR (even Wp): a lane's two columns are
// adjacent in memory, one 8-byte access; odd Wp wraps a pair across the domain edge, two 4-byte ones.
constexpr int TW_W = 128;                // wide region columns (two per lane)

template <bool PAIR, int CP = 0>
__device__ __forceinline__ f32x2 ld2(__amdgpu_buffer_rsrc_t r, int v0, int v1, int soff)
{
    if constexpr (PAIR) {
        const u32x2 x = __builtin_amdgcn_raw_buffer_load_b64(r, v0, soff, CP);
        return f32x2{__uint_as_float(x.x), __uint_as_float(x.y)};
    } else {
        return f32x2{__uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, v0, soff, CP)),
                     __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, v1, soff, CP))};
    }
}
template <bool PAIR, int CP = 0>
__device__ __forceinline__ void st2(f32x2 v, __amdgpu_buffer_rsrc_t r, int v0, int v1, int soff)
{
    if constexpr (PAIR) {
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(v.x), __float_as_uint(v.y)}, r, v0, soff, CP);
    } else {
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v.x), r, v0, soff, CP);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v.y), r, v1, soff, CP);
    }
}

// the four horizontal taps of a column pair c = {x, x+1} (lane shifts; region edges read 0)
struct HTaps { f32x2 l1, r1, l2, r2; };
__device__ __forceinline__ HTaps htaps(f32x2 c)
{
    const float sx = dpp_shr1(c.x), sy = dpp_shr1(c.y), lx = dpp_shl1(c.x), ly = dpp_shl1(c.y);
    HTaps h;
    h.l1 = f32x2{sy, c.x}; h.r1 = f32x2{c.y, lx};
    h.l2 = f32x2{sx, sy};  h.r2 = f32x2{lx, ly};
    return h;
}

// boundary rows 0, 1, R-2, R-1 of every wave through LDS; rows -2, -1, R, R+1 of this wave back
struct Halo2 { f32x2 u2, u1, d1, d2; };
template <int NW, int R>
__device__ __forceinline__ void tw_put(f32x2 (*x)[NW][4][64], int buf, int w, int lane, const f32x2 *v)
{
    x[buf][w][0][lane] = v[0]; x[buf][w][1][lane] = v[1];
    x[buf][w][2][lane] = v[R - 2]; x[buf][w][3][lane] = v[R - 1];
}
template <int NW>
__device__ __forceinline__ Halo2 tw_get(f32x2 (*x)[NW][4][64], int buf, int w, int lane)
{
    const int wu = w > 0 ? w - 1 : 0, wd = w < NW - 1 ? w + 1 : NW - 1;   // (edge waves: halo rows)
    Halo2 h;
    h.u2 = x[buf][wu][2][lane]; h.u1 = x[buf][wu][3][lane];
    h.d1 = x[buf][wd][0][lane]; h.d2 = x[buf][wd][1][lane];
    return h;
}
#define TW_VERT(ARR, r, H2, m2, m1, p1, p2)                                       \
    const f32x2 m2 = (r) >= 2 ? ARR[(r) - 2] : ((r) == 1 ? H2.u1 : H2.u2);        \
    const f32x2 m1 = (r) >= 1 ? ARR[(r) - 1] : H2.u1;                            \
    const f32x2 p1 = (r) + 1 < R ? ARR[(r) + 1] : H2.d1;                         \
    const f32x2 p2 = (r) + 2 < R ? ARR[(r) + 2] : ((r) + 2 == R ? H2.d1 : H2.d2);

// Region geometry shared by the wide kernels (flat locals: uniform values stay SGPRs).
#define TW_REGION_INIT()                                                                           \
    constexpr int H = 2 * T, IW = TW_W - 2 * H, RH = NW * R, IH = RH - 2 * H;                      \
    const TBGeo &g = a.g;                                                                          \
    const int lane = threadIdx.x & 63;                                                             \
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);                                \
    const TileId ti = decode_tile(blockIdx.x, g.tiles_x, g.ntiles, g.B * g.ns_grp);                \
    if (!ti.valid) return;                                          /* whole workgroup: uniform */ \
    const int b = ti.sl / g.ns_grp, s = g.s_off + (ti.sl - b * g.ns_grp), bs = b * g.ns + s;       \
    const int ux = ti.tx * IW - H + 2 * lane;                       /* unwrapped column of .x */   \
    const int gx0 = wrapn(ux, g.Wp), gx1 = wrapn(ux + 1, g.Wp);                                    \
    const bool lin = lane >= H / 2 && lane < 64 - H / 2;            /* interior lane (both cols) */\
    const bool xin0 = lin && ux < g.Wp, xin1 = lin && ux + 1 < g.Wp;                               \
    const int uz0 = ti.ty * IH - H + w * R;                                                        \
    const size_t so = (size_t)bs * g.slice;                                                        \
    const int sbytes = (int)(g.slice * 4);                                                         \
    const int v0 = gx0 * 4, v1 = gx1 * 4;                           /* lane byte offsets in a row */\
    const int vi0 = xin0 ? v0 : OOB, vi1 = xin1 ? v1 : OOB;         /* own (interior) cells only */\
    int rofs[R];                                                    /* wave-uniform gz * ld */     \
    unsigned rin = 0;                                               /* wave-uniform interior rows */\
    _Pragma("unroll") for (int r = 0; r < R; ++r) {                                                \
        const int uz = uz0 + r;                                                                    \
        rofs[r] = wrapn(uz, g.Hp) * g.ld;                                                          \
        const int rr = w * R + r;                                                                  \
        if (rr >= H && rr < RH - H && uz < g.Hp) rin |= 1u << r;                                   \
    }

template <int T, int NW, int R, bool GEN, bool PAIR>
__global__ __launch_bounds__(64 * NW) void k_fwd_tw(FwdTBArgs a)
{
    __shared__ f32x2 xch[2][NW][4][64];
    __shared__ f32x2 As[NW][R][64];      // alpha of the wave's own rows (wave-private), as k_adj_tw
    TW_REGION_INIT()
    // this workgroup's shots: a.spw of the model's shots on one region (k_adj_tw): the coefficients
    // are generated once for all of them
    const int jg = s - g.s_off, s_first = g.s_off + jg * a.spw, nsh = min(a.spw, a.ns_sh - jg * a.spw);
    (void)bs; (void)so;
    f32x2 C1[R], C2v[R];
    unsigned smask = 0;
    int rrow = -1;
    {
        const float *AL = a.coeffs + (size_t)b * g.slice;
        const __amdgpu_buffer_rsrc_t RA = rsrc_of(AL, sbytes), R1 = rsrc_of(AL + g.cstride, sbytes),
                                     R2 = rsrc_of(AL + 2 * g.cstride, sbytes);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int gz = wrapn(uz0 + r, g.Hp);
            if constexpr (GEN) {   // regenerated from the 20 KB-per-row model (L2-resident) instead of 3 fields
                const Coef c0 = gen_coef(a.cg, b, gz, gx0), c1 = gen_coef(a.cg, b, gz, gx1);
                As[w][r][lane] = f32x2{c0.al, c1.al}; C1[r] = f32x2{c0.t1, c1.t1}; C2v[r] = f32x2{c0.t2, c1.t2};
            } else {
                As[w][r][lane] = ld2<PAIR>(RA, v0, v1, rofs[r] * 4);
                C1[r] = ld2<PAIR>(R1, v0, v1, rofs[r] * 4);
                C2v[r] = ld2<PAIR>(R2, v0, v1, rofs[r] * 4);
            }
            if (gz == g.isz) smask |= 1u << r;          // (tiny domains: a wave can hold the row twice)
            if (gz == g.igz) rrow = r;
        }
    }
    // receivers of the lane's two columns (usually one each), read once
    int rs0 = 0, re0 = 0, rs1 = 0, re1 = 0;
    if (rrow >= 0) { rs0 = g.rcv_start[gx0]; re0 = g.rcv_start[gx0 + 1]; rs1 = g.rcv_start[gx1]; re1 = g.rcv_start[gx1 + 1]; }
    const int rc0 = xin0 && rs0 < re0 ? g.rcv_list[rs0] : -1, rc1 = xin1 && rs1 < re1 ? g.rcv_list[rs1] : -1;
    const bool rmulti = __any(re0 - rs0 > 1 || re1 - rs1 > 1);   // wave-uniform
    const f32x2 kC2 = {C2, C2}, kC3 = {C3, C3};
    // kernel arguments re-read from the kernarg segment per shot (k_adj_tw); a shot's two input levels
    // are loaded when the previous shot's last levels have been stored (k_adj_tw's pipelining)
    auto kargs = [&]() {
        const __attribute__((address_space(4))) FwdTBArgs *k_ =
            (const __attribute__((address_space(4))) FwdTBArgs *)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(k_));
        return k_;
    };
    f32x2 P0[R], P1[R];
    auto load_shot = [&](int ss_) {
        const auto *k_ = kargs();
        const size_t so_ = (size_t)(b * k_->g.ns + ss_) * k_->g.slice;
        const __amdgpu_buffer_rsrc_t RPv = rsrc_of(k_->in_prev + so_, sbytes), RCu = rsrc_of(k_->in_cur + so_, sbytes);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            P0[r] = ld2<PAIR>(RPv, v0, v1, rofs[r] * 4);
            P1[r] = ld2<PAIR>(RCu, v0, v1, rofs[r] * 4);
        }
    };
    load_shot(s_first);
    for (int sh = 0; sh < nsh; ++sh) {
    const auto *ka = kargs();
    const int ss = s_first + sh, bss = b * ka->g.ns + ss;
    const size_t soo = (size_t)bss * ka->g.slice;
    // an odd T ends on exchange buffer 0, which the next shot's first step rewrites: wait for every
    // wave's last halo reads (an even T ends on buffer 1, and buffer 0's last reads precede the last
    // step's barrier)
    if ((T & 1) && sh) __syncthreads();
    const int isx = ka->g.isx[ss];
    const bool sc0 = gx0 == isx, sc1 = gx1 == isx;
    const float bsrc = smask ? ka->coeffs[4 * ka->g.cstride + (size_t)b * ka->g.slice + (size_t)ka->g.isz * ka->g.ld + isx] : 0.0f;
#pragma unroll
    for (int t = 0; t < T; ++t) {       // exactly T steps (the host launches a shorter tail as its own T)
        f32x2 *cur = (t & 1) ? P0 : P1;     // P_{n+t}
        f32x2 *prv = (t & 1) ? P1 : P0;     // P_{n+t-1} -> P_{n+t+1}
        tw_put<NW, R>(xch, t & 1, w, lane, cur);
        __syncthreads();
        const Halo2 h2 = tw_get<NW>(xch, t & 1, w, lane);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            TW_VERT(cur, r, h2, zm2, zm1, zp1, zp2)
            const f32x2 c = cur[r];
            const HTaps x = htaps(c);
            // pde.py:79, reference evaluation order per cell
            f32x2 s1 = zm1 + zp1; s1 = s1 + x.l1; s1 = s1 + x.r1;
            f32x2 s2 = zm2 + zp2; s2 = s2 + x.l2; s2 = s2 + x.r2;
            f32x2 lap = kC2 * s1; const f32x2 l2 = kC3 * s2; lap = lap + l2;
            f32x2 a1 = C1[r] * c; const f32x2 a2 = C2v[r] * prv[r]; a1 = a1 - a2;
            const f32x2 a3 = As[w][r][lane] * lap;
            prv[r] = a1 + a3;
        }
        if (smask) {                                                   // pde.py:80-81
            const float add = bsrc * ka->w[t];
            const f32x2 av = {sc0 ? add : -0.0f, sc1 ? add : -0.0f};   // x + (-0) == x bit for bit
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (smask & (1u << r)) prv[r] = prv[r] + av;
        }
        const int n = ka->n0 + t;
        if (ka->hist) {
            const __amdgpu_buffer_rsrc_t HS = rsrc_of(ka->hist + (size_t)(n + 2) * ka->g.level + soo, sbytes);
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (rin & (1u << r)) st2<PAIR, CP_NT>(prv[r], HS, vi0, vi1, rofs[r] * 4);   // streaming
        }
        if (rrow >= 0 && (rin & (1u << rrow)) && (n % ka->g.st) == 0) {   // pde.py:82-83
            f32x2 val = prv[0];
#pragma unroll
            for (int r = 1; r < R; ++r) if (r == rrow) val = prv[r];
            float *SK = ka->seis + ((size_t)bss * ka->g.nrec + n / ka->g.st) * ka->g.ng;
            if (rc0 >= 0) SK[rc0] = val.x;
            if (rc1 >= 0) SK[rc1] = val.y;
            if (rmulti) {
                if (xin0) for (int j = rs0 + 1; j < re0; ++j) SK[ka->g.rcv_list[j]] = val.x;
                if (xin1) for (int j = rs1 + 1; j < re1; ++j) SK[ka->g.rcv_list[j]] = val.y;
            }
        }
    }
    if (ka->out_cur) {   // ring path: keep the last two levels
        constexpr bool odd = (T & 1) != 0;      // after T steps the newest level is in P0 if odd
        const __amdgpu_buffer_rsrc_t OC = rsrc_of(ka->out_cur + soo, sbytes), OP = rsrc_of(ka->out_prev + soo, sbytes);
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (rin & (1u << r)) {
                st2<PAIR>(odd ? P0[r] : P1[r], OC, vi0, vi1, rofs[r] * 4);
                st2<PAIR>(odd ? P1[r] : P0[r], OP, vi0, vi1, rofs[r] * 4);
            }
    }
    if (sh + 1 < nsh) load_shot(ss + 1);
    }   // shots
}

// Adjoint on wide regions (k_adj_tb's per-cell arithmetic):
//   L_k = T1 L_{k+1} - T2 L_{k+2} + (c2 N1(A L_{k+1}) + c3 N2(A L_{k+1})) [+ R^T dseis[k-1]]
//   gA_s += L_k (2c1 P_{k-1} + c2 S1(P_{k-1}) + c3 S2(P_{k-1})),  gk += (K P_{k-1})(L_{k+1} - L_k)
//   gbeta[s] += L_k(src) w[k-1]           (own cells; gA loaded and stored once per launch)
// EXACT: the oracle's fp32 operation order (bitwise gA / gbeta).  Else the same stencils with FMA
// contraction (fp32-level tolerance: rdq_fwi_set_variant without RDQ_VARIANT_ADJ_EXACT, nbc >= 20).
// Every gk term is summed in fp64 in both.  alpha and kappa are
// regenerated from the model in registers (gen_coef, bit-identical to K3's fields): the 16 shots of a
// tile then read the L2-resident 6 MB model instead of two padded fields each.  Loads are issued in
// the order the first step uses them (alpha's model values and L_{k+1} first).
template <int T, int NW, int R, bool PAIR, bool EXACT>
__global__ __launch_bounds__(64 * NW) void k_adj_tw(AdjTBArgs a)
{
    __shared__ f32x2 xq[2][NW][4][64];
    __shared__ f32x2 xp[2][NW][4][64];
    __shared__ f32x2 As[NW][R][64];      // alpha of the wave's own rows (wave-private: no barrier), in LDS
                                         // instead of 8 VGPRs live across the shot loop
    TW_REGION_INIT()
    // this workgroup's shots: group jg of the model's shots (a.spw each), all on the same region, so
    // alpha / kappa are generated once for all of them (~10 ms of the adjoint at configs[4] when every
    // shot's workgroup generated its own: profiles/r5/configs4_adj_coef_ab.jsonl)
    const int jg = s - g.s_off, s_first = g.s_off + jg * a.spw, nsh = min(a.spw, a.ns_sh - jg * a.spw);
    (void)bs; (void)so;
    f32x2 KP[R];                         // temp1 / temp2 re-derived per step (bit-identical)
    unsigned pmask = 0, smask = 0, rmask = 0;            // wave-uniform row masks
    const f32x2 kC2 = {C2, C2}, kC3 = {C3, C3}, kC1X2 = {C1X2, C1X2}, k2 = {2.0f, 2.0f}, k1 = {1.0f, 1.0f};
    // history P_{k-1}: only the columns the own cells' gradient stencil reaches (own +- 2: lanes H/2 - 1
    // .. 64 - H/2), the other halo lanes' loads are out of range (no memory access, zeros): 112 of 128
    // columns at T = 5, the history being the adjoint's largest stream
    const bool plane = lane >= H / 2 - 1 && lane < 64 - H / 2 + 1;
    const int pv0 = plane ? v0 : OOB, pv1 = plane ? v1 : OOB;
    {
        int gz[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            gz[r] = wrapn(uz0 + r, g.Hp);
            const int rr = w * R + r;
            if (rr >= H - 2 && rr < RH - H + 2) pmask |= 1u << r;
            if (gz[r] == g.isz) smask |= 1u << r;
            if (gz[r] == g.igz) rmask |= 1u << r;
        }
        Coef c0[R], c1[R];
#pragma unroll
        for (int r = 0; r < R; ++r) { c0[r] = gen_coef(a.cg, b, gz[r], gx0); c1[r] = gen_coef(a.cg, b, gz[r], gx1); }
#pragma unroll
        for (int r = 0; r < R; ++r) { As[w][r][lane] = f32x2{c0[r].al, c1[r].al}; KP[r] = f32x2{c0[r].kp, c1[r].kp}; }
    }
    const int rcv0 = rmask ? g.rlane[gx0] : -1, rcv1 = rmask ? g.rlane[gx1] : -1;
    // a shot's launch-start loads (levels L_{k0+1}, L_{k0+2}, history P_{k0-1}, gA): shot 0's here,
    // shot s+1's right after shot s's output stores, so they are in flight during shot s's gk
    // reduction.  Kernel arguments are re-read from the kernarg segment (an opaque pointer) per
    // shot: kept live across the shot loop they exhaust the SGPRs and spill.
    f32x2 L0[R], L1[R], GA[R], Pn[R];
    auto kargs = [&]() {
        const __attribute__((address_space(4))) AdjTBArgs *k_ =
            (const __attribute__((address_space(4))) AdjTBArgs *)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(k_));
        return k_;
    };
    auto load_shot = [&](int ss_) {
        const auto *k_ = kargs();
        const size_t so_ = (size_t)(b * k_->g.ns + ss_) * k_->g.slice;
        const __amdgpu_buffer_rsrc_t RL1 = rsrc_of(k_->in_l1 + so_, sbytes), RL2 = rsrc_of(k_->in_l2 + so_, sbytes);
        const __amdgpu_buffer_rsrc_t RG = rsrc_of(k_->gA + so_, sbytes);
        const __amdgpu_buffer_rsrc_t HR = rsrc_of(k_->hist + (size_t)k_->k0 * k_->g.level + so_, sbytes);
#pragma unroll
        for (int r = 0; r < R; ++r) L1[r] = ld2<PAIR>(RL1, v0, v1, rofs[r] * 4);   // L_{k+1}
#pragma unroll
        for (int r = 0; r < R; ++r) L0[r] = ld2<PAIR>(RL2, v0, v1, rofs[r] * 4);   // L_{k+2}
#pragma unroll
        for (int r = 0; r < R; ++r) Pn[r] = (pmask & (1u << r)) ? ld2<PAIR>(HR, pv0, pv1, rofs[r] * 4) : f32x2{0.0f, 0.0f};
#pragma unroll
        for (int r = 0; r < R; ++r) GA[r] = (rin & (1u << r)) ? ld2<PAIR>(RG, vi0, vi1, rofs[r] * 4) : f32x2{0.0f, 0.0f};
    };
    load_shot(s_first);
    for (int sh = 0; sh < nsh; ++sh) {
    const auto *ka = kargs();
    const int ss = s_first + sh, bss = b * ka->g.ns + ss;
    const size_t soo = (size_t)bss * ka->g.slice;
    // (no barrier between shots: the gk reduction's LDS words are wave 0's own exchange slot, which
    //  only wave 0 rewrites, after its thread 0 has read them; the reduction's two barriers order the
    //  last step's halo reads before the next shot's first exchange)
    const int isx = ka->g.isx[ss];
    const bool sc0 = xin0 && gx0 == isx, sc1 = xin1 && gx1 == isx;   // the source cell is an own cell
    const __amdgpu_buffer_rsrc_t DSR = rsrc_of(ka->dseis + (size_t)bss * ka->g.nrec * ka->g.dstride);
    const bool gbl = (smask & rin) && (sc0 || sc1);
    float gbacc = gbl ? ka->gbeta[bss] : 0.0f;
    double ksum = 0.0;                   // every gk term in fp64
#pragma unroll
    for (int t = 0; t < T; ++t) {       // exactly T steps (the host launches a shorter tail as its own T)
        __builtin_amdgcn_sched_barrier(0);  // no step's work moved into another (live ranges: no spills)
        const int k = ka->k0 - t;
        f32x2 *cur = (t & 1) ? L0 : L1;     // L_{k+1}
        f32x2 *prv = (t & 1) ? L1 : L0;     // L_{k+2} -> L_k
        f32x2 P[R];
#pragma unroll
        for (int r = 0; r < R; ++r) P[r] = Pn[r];
        if (t + 1 < T) {   // history P_{k-2} of the next step, on the rows the interior's stencil needs
            const __amdgpu_buffer_rsrc_t HR = rsrc_of(ka->hist + (size_t)(k - 1) * ka->g.level + soo, sbytes);
#pragma unroll
            for (int r = 0; r < R; ++r) if (pmask & (1u << r)) Pn[r] = ld2<PAIR>(HR, pv0, pv1, rofs[r] * 4);
        }
        // this step's receiver residuals, loaded before the stencil so their latency hides under it
        const int ri = rmask ? rec_index(k - 1, ka->g.st) : -1;   // wave-uniform
        f32x2 dsv = {-0.0f, -0.0f};
        if (ri >= 0) {
            const int ro = ri * ka->g.dstride;
            const float d0 = bload(DSR, rcv0 >= 0 ? (ro + rcv0) * 4 : OOB, 0);
            const float d1 = bload(DSR, rcv1 >= 0 ? (ro + rcv1) * 4 : OOB, 0);
            dsv = f32x2{rcv0 >= 0 ? d0 : -0.0f, rcv1 >= 0 ? d1 : -0.0f};
        }
        f32x2 q[R];
#pragma unroll
        for (int r = 0; r < R; ++r) q[r] = As[w][r][lane] * cur[r];
        tw_put<NW, R>(xq, t & 1, w, lane, q);
        tw_put<NW, R>(xp, t & 1, w, lane, P);
        __syncthreads();
        const Halo2 hq = tw_get<NW>(xq, t & 1, w, lane);
        const Halo2 hp = tw_get<NW>(xp, t & 1, w, lane);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            TW_VERT(q, r, hq, qm2, qm1, qp1, qp2)
            const HTaps x = htaps(q[r]);
            f32x2 n1 = qm1 + qp1; n1 = n1 + x.l1; n1 = n1 + x.r1;
            f32x2 n2 = qm2 + qp2; n2 = n2 + x.l2; n2 = n2 + x.r2;
            if constexpr (EXACT) {
                f32x2 nb = kC2 * n1; const f32x2 nb2 = kC3 * n2; nb = nb + nb2;
                f32x2 t1 = kC1X2 * As[w][r][lane]; t1 = t1 + k2; t1 = t1 - KP[r];      // pde.py:69
                const f32x2 t2 = k1 - KP[r];                                  // pde.py:70
                f32x2 l = t1 * cur[r]; const f32x2 l2 = t2 * prv[r]; l = l - l2; l = l + nb;
                prv[r] = l;
            } else {
                const f32x2 nb = fma2(kC3, n2, kC2 * n1);
                const f32x2 t1 = fma2(kC1X2, As[w][r][lane], k2) - KP[r], t2 = k1 - KP[r];
                prv[r] = fma2(t1, cur[r], fma2(-t2, prv[r], nb));
            }
        }
        if (ri >= 0) {                          // adjoint of the receiver sampling
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (rmask & (1u << r)) prv[r] = prv[r] + dsv;      // -0 on lanes without a receiver
        }
        // gradient accumulators (own cells are the ones stored; halo lanes compute and discard)
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (!(rin & (1u << r))) continue;   // wave-uniform
            TW_VERT(P, r, hp, pm2, pm1, pp1, pp2)
            const f32x2 pc = P[r];
            const HTaps x = htaps(pc);
            f32x2 s1 = pm1 + pp1; s1 = s1 + x.l1; s1 = s1 + x.r1;
            f32x2 s2 = pm2 + pp2; s2 = s2 + x.l2; s2 = s2 + x.r2;
            const f32x2 l = prv[r];
            const f32x2 dl = cur[r] - l;
            if constexpr (EXACT) {
                f32x2 lap = kC2 * s1; const f32x2 lq = kC3 * s2; lap = lap + lq;
                f32x2 d = kC1X2 * pc; d = d + lap;
                const f32x2 c = l * d;
                GA[r] = GA[r] + c;
                f32x2 kk = KP[r] * pc; kk = kk * dl;                      // fp32 term, fp64 sum
                ksum += xin0 ? (double)kk.x : 0.0;
                ksum += xin1 ? (double)kk.y : 0.0;
            } else {
                const f32x2 d = fma2(kC1X2, pc, fma2(kC3, s2, kC2 * s1));
                GA[r] = fma2(l, d, GA[r]);
                const f32x2 kk = (KP[r] * pc) * dl;                    // fp32 term, fp64 sum (the total
                ksum += (double)(xin0 ? kk.x : 0.0f);                   //  cancels: fp32 partials lost
                ksum += (double)(xin1 ? kk.y : 0.0f);                   //  1.3e-4 of it at OpenFWI)
            }
            if ((smask & (1u << r)) && (sc0 || sc1)) { const float gb = (sc0 ? l.x : l.y) * ka->w[t]; gbacc = gbacc + gb; }
        }
    }
    {
        constexpr bool odd = (T & 1) != 0;      // newest level (L_{k0-T+1}) is in L0 if odd
        const __amdgpu_buffer_rsrc_t O1 = rsrc_of(ka->out_l1 + soo, sbytes), O2 = rsrc_of(ka->out_l2 + soo, sbytes);
        const __amdgpu_buffer_rsrc_t RG = rsrc_of(ka->gA + soo, sbytes);
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (rin & (1u << r)) {
                st2<PAIR>(odd ? L0[r] : L1[r], O1, vi0, vi1, rofs[r] * 4);
                st2<PAIR>(odd ? L1[r] : L0[r], O2, vi0, vi1, rofs[r] * 4);
                st2<PAIR>(GA[r], RG, vi0, vi1, rofs[r] * 4);
            }
    }
    if (sh + 1 < nsh) load_shot(ss + 1);
    if (gbl) ka->gbeta[bss] = gbacc;
    // deterministic workgroup reduction of the sponge-coefficient partial sum: a fixed xor tree per
    // wave, then the NW wave sums in wave order (LDS of the exchange)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ksum += __shfl_xor(ksum, o, 64);
    double *red = reinterpret_cast<double *>(&xq[0][0][0][0]);
    __syncthreads();
    if (lane == 0) red[w] = ksum;
    __syncthreads();
    if (threadIdx.x == 0) {
        double tot = red[0];
        for (int i = 1; i < NW; ++i) tot += red[i];
        // one add per (slot, launch), launches in stream order: the same sum as a load-add-store, but
        // without the load's round trip before the next shot's barrier
        unsafeAtomicAdd(&ka->gk_part[(size_t)bss * ka->nblk + ti.tile], tot);
    }
    }   // shots
}
#undef TW_VERT
#undef TW_REGION_INIT

// --------------------------------------------------------------------------------------- K1/K2
// Persistent variants: ONE launch runs the whole time loop.  Every workgroup keeps its region
// (coefficients + two wavefield levels) in VGPRs for all nt steps; after each epoch of T steps it
// publishes the H-wide border of its interior (the only cells any other region's halo reads) and
// reloads its own halo ring from the neighbours' publications.  The hand-off is the
// data-is-the-flag form (8-byte {tag, value} granules, write-through `sc1` stores, `sc1` loads
// re-read until every tag matches: cdna_hip_programming.md §6 G16, R2), so there is no flag, no
// fence and no kernel boundary between epochs — the per-launch prologue, store drain and launch gap
// of the chunked path (≈7.5 µs per forward launch at OpenFWI size) become one hand-off per epoch.
// Needs every workgroup of the launch resident at once: the host checks the grid against the
// occupancy query and uses the chunked kernels otherwise; every spin is bounded (a timeout sets
// the plan's status word, reported by rdq_fwi_status, and the kernel still runs to completion).
//
// The time step is VALU-issue-bound (wave64 fp32 VALU = 4 cycles), so the kernels are written
// to keep per-cell instructions at the stencil's own: row predicates are wave-uniform bits, the
// per-lane ones are three loop-invariant masks, and every history / granule access is a buffer
// instruction (scalar base + one lane offset + one uniform row offset: no 64-bit address VALU).
// Region height is a template parameter (NW waves x 8 rows): 12 waves -> 64 x 96 regions, one
// workgroup per CU at OpenFWI size (28 tiles x 8 shots = 224 <= 256 CUs).
//
// Granule buffer (inside the caller's `ring`): [2 epoch parity][B][ns][Hp][ld] x 16-B granules,
// zeroed before each launch; tag = epoch index (>= 1) so a zeroed granule never matches.
constexpr int CP_SC1 = 16;                            // buffer cache policy: sc1 (write-through / L1 bypass)
constexpr int PT_ADJ_SG = 8;                          // adjoint hand-off sweep: rows per load group
constexpr size_t PROF_RAW = 8;                        // per-wave records after the 4 summary words
constexpr size_t PROF_WAVES = 4096 * 16;              // blocks x waves recorded
constexpr size_t PROF_WORDS = PROF_RAW + PROF_WAVES * 3;   // per kernel (fwd, then adj)
constexpr unsigned long long PT_TIMEOUT_TICKS = 20000000ull;   // 200 ms of s_memrealtime (100 MHz)

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
// One cell's hand-off granule = BOTH wavefield levels, 16 bytes {v0, tag, v1, tag}: each 8-byte
// half carries its own epoch tag, so a read torn between the halves is still caught by the tag
// check (the guarantee used is only that an aligned 8-byte store is seen whole), and a sweep or a
// publish is one dwordx4 instruction per row instead of two dwordx2.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u32x4 gran2(unsigned tag, float v0, float v1)
{
    u32x4 x;
    x.x = __float_as_uint(v0); x.y = tag; x.z = __float_as_uint(v1); x.w = tag;
    return x;
}
__device__ __forceinline__ void gran_put(__amdgpu_buffer_rsrc_t r, int voff, int soff, unsigned tag, float v0, float v1)
{
    __builtin_amdgcn_raw_buffer_store_b128(gran2(tag, v0, v1), r, voff, soff, CP_SC1);
}
// XCD-local hand-off: a plain store stays in the producer XCD's L2, where a same-XCD consumer's
// sc1 (L1-bypassing, L2-served) load sees it without the write-through round trip to memory
// (tools/probe/l2_probe.hip)
__device__ __forceinline__ void gran_put_l2(__amdgpu_buffer_rsrc_t r, int voff, int soff, unsigned tag, float v0, float v1)
{
    __builtin_amdgcn_raw_buffer_store_b128(gran2(tag, v0, v1), r, voff, soff, 0);
}
__device__ __forceinline__ u32x4 gran_get(__amdgpu_buffer_rsrc_t r, int voff, int soff)
{
    return __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, CP_SC1);
}

// A wavelet sample at a wave-uniform step, read through the scalar cache (s_load into an SGPR): out of
// the vector memory queue, where, with gfx9's in-order vmcnt, the forward's source row waited for its
// next epoch's samples behind the deferred history stores.  Forward: issued right after the publish,
// 1.362 -> 1.334 ms at configs[1] (profiles/r6/wav_scalar_ab.txt); the adjoint keeps vector loads.
__device__ __forceinline__ float wav_s(const float *w, int i)
{
    return ((const __attribute__((address_space(4))) float *)w)[i];
}

// padded-grid row of region row uz (periodic wrap, pde.py:79); |uz| < 2 Hp
__device__ __forceinline__ int wrap_row(int uz, int Hp)
{
    uz = uz < 0 ? uz + Hp : uz;
    return uz >= Hp ? uz - Hp : uz;
}

// Slice / tile assignment of a persistent launch by the XCD each workgroup actually runs on.
// Every workgroup reads its XCD id (s_getreg HW_REG_XCC_ID), takes a slot on that XCD's arrival
// counter and waits until all gridDim.x workgroups have arrived (the launch is fully resident by
// construction: the host sizes the grid to the occupancy query).  From the final per-XCD counts
// every workgroup derives the same assignment: whole (model, shot) slices go to single XCDs in XCD
// order ("local" slices: every hand-off between their tiles stays inside one L2, so granules are
// published with plain stores that stay in that L2); slices that do not fit whole on one XCD are
// dealt over the leftover workgroups ("global": write-through sc1 granules, as before).
// Correctness never depends on the placement guess: the XCD id is read, not assumed, and every
// granule carries its epoch tag, so a stale read is re-polled, never consumed.
struct PtTile { int tx, ty, tile, sl; bool valid, local; };
constexpr unsigned long long PT_ARRIVE_TICKS = 10000000ull;   // 100 ms

__device__ PtTile pt_assign(const TBGeo &g, unsigned *status, int xcd_mode)
{
    __shared__ int sh[3];
    unsigned *cnt = status + 16;                         // [8] per-XCD arrivals (zeroed per launch)
    if (threadIdx.x == 0) {
        unsigned x = 0;
        if (xcd_mode) {
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
            x &= 7u;
        }
        const unsigned slot = __hip_atomic_fetch_add(cnt + x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned n[8], tot = 0;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        bool ok = true;
        for (;;) {
            tot = 0;
            for (int i = 0; i < 8; ++i) {
                n[i] = __hip_atomic_load(cnt + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                tot += n[i];
            }
            if (tot >= gridDim.x) break;
            if (__builtin_amdgcn_s_memrealtime() - t0 > PT_ARRIVE_TICKS) { ok = false; break; }
            __builtin_amdgcn_s_sleep(2);
        }
        int sl = -1, tile = 0, local = 0;
        if (ok) {
            const int Tt = g.ntiles, S = g.nsl;
            int placed = 0, take[8];
            for (int i = 0; i < 8; ++i) {
                take[i] = xcd_mode ? min((int)n[i] / Tt, S - placed) : 0;
                placed += take[i];
            }
            int base = 0;
            for (int i = 0; i < (int)x; ++i) base += take[i];
            if ((int)slot < take[x] * Tt) {
                sl = base + (int)slot / Tt; tile = (int)slot % Tt; local = 1;
            } else {
                int r = (int)slot - take[x] * Tt;
                for (int i = 0; i < (int)x; ++i) r += (int)n[i] - take[i] * Tt;
                if (r < (S - placed) * Tt) { sl = placed + r / Tt; tile = r % Tt; }
            }
        } else {
            __hip_atomic_store(status, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // not resident
        }
        sh[0] = sl; sh[1] = tile; sh[2] = local;
    }
    __syncthreads();
    PtTile t;
    t.sl = sh[0]; t.tile = sh[1]; t.local = sh[2] != 0;
    t.valid = t.sl >= 0;
    t.ty = t.tile / g.tiles_x;
    t.tx = t.tile - t.ty * g.tiles_x;
    return t;
}

// Region geometry of the persistent kernels (flat locals so every block-/wave-uniform value stays
// provably uniform: SGPRs and scalar branches, never waterfall loops).  Row classes are
// wave-uniform bit masks; lane classes: xin (own interior column), bx (interior column within H of
// the tile's x edge, or a one-tile-wide grid), cx (column within H of the own interior: the
// T-step dependence cone).
#define PT_REGION_INIT(NW_, RW_)                                                                    \
    PT_REGION_HEAD(NW_, RW_)                                                                        \
    const int bs = __builtin_amdgcn_readfirstlane(g.sl_off + ti.sl);                                \
    const int b = __builtin_amdgcn_readfirstlane(bs / g.ns);                                        \
    const int s = __builtin_amdgcn_readfirstlane(bs - b * g.ns);                                    \
    PT_REGION_GEOM()

// Workgroup placement (pt_assign: a (slice, tile) of the launch) and the region's constants
#define PT_REGION_HEAD(NW_, RW_)                                                                    \
    constexpr int R = (RW_), RP = (RW_) / 2, RH = (NW_) * (RW_), H = 2 * T, IW = 64 - 2 * H,       \
                  IH = RH - 2 * H;                                                                  \
    const int lane = threadIdx.x & 63;                                                              \
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);                                \
    const PtTile ti = pt_assign(g, a.status, a.xcd_mode);                                           \
    if (!ti.valid) return;                                                                          \
    const bool gl2 = ti.local;                     /* uniform: XCD-local slice, L2 hand-offs */

// The slice-independent part of PT_REGION_INIT (`bs` = the workgroup's flat (model, shot) slice)
#define PT_REGION_GEOM()                                                                            \
    const int tx = __builtin_amdgcn_readfirstlane(ti.tx), ty = __builtin_amdgcn_readfirstlane(ti.ty); \
    const int tile = __builtin_amdgcn_readfirstlane(ti.tile);                                       \
    const int ux = tx * IW - H + lane;                                                              \
    const int gx = wrapn(ux, g.Wp);                                                                 \
    const bool xin = lane >= H && lane < 64 - H && ux < g.Wp;                                       \
    const int vw = min(IW, g.Wp - tx * IW), vh = min(IH, g.Hp - ty * IH);                           \
    const bool bx = g.tiles_x == 1 || lane - H < H || lane - H >= vw - H;                           \
    const bool cx = lane - H < vw + H;                                                              \
    const int uz0 = ty * IH - H + w * R;                                                            \
    unsigned rin = 0, rby = 0, rcy = 0;                                                             \
    _Pragma("unroll") for (int r = 0; r < R; ++r) {                                                 \
        const int rr = w * R + r, ly = rr - H;                                                      \
        if (rr >= H && rr < RH - H && uz0 + r < g.Hp) rin |= 1u << r;                               \
        if (g.ntiles == g.tiles_x || ly < H || ly >= vh - H) rby |= 1u << r;                        \
        if (ly < vh + H) rcy |= 1u << r;                                                            \
    }                                                                                               \
    const size_t so = (size_t)bs * g.slice;                                                         \
    const int vo16 = gx * 16;                                                                       \
    const bool hx = !xin && cx, xb = xin && bx;                                                     \
    /* hand-off lane offsets (OOB: no access) */                                                    \
    const int vo_hx = hx ? vo16 : OOB, vo_cx = cx ? vo16 : OOB;                                     \
    const int vo_xin = xin ? vo16 : OOB, vo_xb = xb ? vo16 : OOB;                                   \
    const bool keep_in = xin || cx;
#define PT_ROFS(r) (wrap_row(uz0 + (r), g.Hp) * g.ld)

// Reload the halo cells of two levels V0/V1 from the granule slot GR (16-byte two-level granules),
// zero the dead cells.  `live` turns false once this wave gave up (timeout / another's timeout).
// The wave's own traffic for the next epoch (history stores / prefetch loads, wavelet, receiver
// residuals) is issued only AFTER the sweep (FWD_ISSUE / ADJ_ISSUE), not before it: a hand-off's
// latency is set by the consumer CU's own memory queue (MI355X_MICROARCH.md, handoff-1to1), and on
// gfx9 the in-order vmcnt also counts stores, so the granule loads would otherwise wait behind it.
#define PT_SWEEP(GR, TAG, V0, V1, SG)                                                               \
    {                                                                                               \
        unsigned long long t0_ = 0;                                                                 \
        const unsigned long long ts_ = prof ? __builtin_amdgcn_s_memrealtime() : 0;                 \
        if constexpr (PT_PRIO) __builtin_amdgcn_s_setprio(PT_PRIO_WAIT);                            \
        for (unsigned pass_ = 0; live; ++pass_) {                                                   \
            /* the loads of a group of SG rows are all issued before any is checked: lanes        \
               without a halo cell in a row load from an out-of-range offset (no memory access,   \
               returns 0) instead of branching, which would make the compiler wait vmcnt(0) after \
               each load (one serial L2 round trip per row).  SG < R bounds the registers held.   \
               The row classes are laundered per pass so no per-row lane mask stays live (SGPR    \
               pressure) across the time loop.                                                    */ \
            unsigned rin_ = rin, rcy_ = rcy;                                                        \
            LAUNDER(rin_); LAUNDER(rcy_);                                                           \
            bool ok_ = true;                                                                        \
            _Pragma("unroll") for (int g_ = 0; g_ < R; g_ += (SG)) {                                \
                u32x4 x_[(SG)];                                                                     \
                int o_[(SG)];                                                                       \
                constexpr int GN_ = (SG) < R ? (SG) : R;   /* SG need not divide R: rows past R skipped */ \
                _Pragma("unroll") for (int i_ = 0; i_ < GN_; ++i_) {                                \
                    const int r = g_ + i_ < R ? g_ + i_ : R - 1;                                    \
                    const bool rowin_ = g_ + i_ < R && ((rin_ >> r) & 1u), rowcy_ = g_ + i_ < R && ((rcy_ >> r) & 1u); \
                    o_[i_] = rowin_ ? vo_hx : (rowcy_ ? vo_cx : OOB);                               \
                    x_[i_] = gran_get(GR, o_[i_], PT_ROFS(r) * 16);                                 \
                }                                                                                   \
                _Pragma("unroll") for (int i_ = 0; i_ < GN_; ++i_) {                                \
                    const int r = g_ + i_ < R ? g_ + i_ : R - 1;                                    \
                    const bool nd_ = o_[i_] != OOB;                                                 \
                    ok_ = ok_ && (!nd_ || (x_[i_].y == (TAG) && x_[i_].w == (TAG)));                \
                    PT_AT(V0, r) = nd_ ? __uint_as_float(x_[i_].x) : PT_AT(V0, r);                  \
                    PT_AT(V1, r) = nd_ ? __uint_as_float(x_[i_].z) : PT_AT(V1, r);                  \
                }                                                                                   \
            }                                                                                       \
            const bool done_ = __all(ok_);                                                          \
            if (prof && pass_ == 0) tfp += __builtin_amdgcn_s_memrealtime() - ts_;                   \
            if (done_) { npass += pass_ + 1; break; }                                               \
            if (pass_ == 0) t0_ = __builtin_amdgcn_s_memrealtime();                                 \
            if ((pass_ & 15) == 15) {                                                               \
                if (__hip_atomic_load(a.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)   \
                    live = false;                                                                   \
                else if (__builtin_amdgcn_s_memrealtime() - t0_ > PT_TIMEOUT_TICKS) {               \
                    __hip_atomic_store(a.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   \
                    if (lane == 0) {                    /* diagnostics: rdq_fwi_debug_words */      \
                        a.status[1] = (TAG); a.status[2] = blockIdx.x; a.status[3] = bs;            \
                        a.status[4] = tile; a.status[5] = gl2; a.status[6] = w;                      \
                    }                                                                               \
                    live = false;                                                                   \
                }                                                                                   \
            }                                                                                       \
            __builtin_amdgcn_s_sleep(1);                                                            \
        }                                                                                           \
        if constexpr (PT_PRIO) __builtin_amdgcn_s_setprio(PT_PRIO_SWEPT);                           \
        /* cells outside the next epoch's dependence cone: zeroed (bounded garbage) */             \
        unsigned rin_ = rin, rcy_ = rcy;                                                            \
        LAUNDER(rin_); LAUNDER(rcy_);                                                               \
        _Pragma("unroll") for (int r = 0; r < R; ++r) {                                             \
            const bool rowin_ = (rin_ >> r) & 1u, rowcy_ = (rcy_ >> r) & 1u;                        \
            const bool keep_ = rowin_ ? keep_in : (rowcy_ && cx);                                   \
            PT_AT(V0, r) = keep_ ? PT_AT(V0, r) : 0.0f;                                             \
            PT_AT(V1, r) = keep_ ? PT_AT(V1, r) : 0.0f;                                             \
        }                                                                                           \
    }

// publish the own-interior border cells of two levels (rows: interior; lanes: the interior
// columns of border rows, else the border columns)
#define PT_PUBLISH(GR, TAG, V0, V1)                                                                 \
    {                                                                                               \
        unsigned rin_ = rin, rby_ = rby;                                                            \
        LAUNDER(rin_); LAUNDER(rby_);                                                               \
        if (gl2) {                                                                                  \
            _Pragma("unroll") for (int r = 0; r < R; ++r) {                                         \
                if (!((rin_ >> r) & 1u)) continue;                                                  \
                gran_put_l2(GR, ((rby_ >> r) & 1u) ? vo_xin : vo_xb, PT_ROFS(r) * 16, (TAG),        \
                            PT_AT(V0, r), PT_AT(V1, r));                                            \
            }                                                                                       \
        } else {                                                                                    \
            _Pragma("unroll") for (int r = 0; r < R; ++r) {                                         \
                if (!((rin_ >> r) & 1u)) continue;                                                  \
                gran_put(GR, ((rby_ >> r) & 1u) ? vo_xin : vo_xb, PT_ROFS(r) * 16, (TAG),           \
                         PT_AT(V0, r), PT_AT(V1, r));                                               \
            }                                                                                       \
        }                                                                                           \
    }

// The first hand-off pass of an epoch is issued `a.sweep_delay` ticks after the wave's publish: a pass
// issued at once mostly finds the neighbours' granules not yet there (1.9 passes per epoch, each an L2
// round trip of ~0.7 us) and a failed pass's loads sit in the CU's memory queue ahead of the next
// pass's.  Measured at configs[1] (profiles/r6/sweep_delay_*): 0.25 us takes the forward 1.371 ->
// 1.321 ms and the adjoint 1.688 -> 1.647 ms; 1 us is flat, 2 us slower.  With the wave priorities and
// the barrier-free adjoint (profiles/r6/delay_retune_ab.txt): forward best at 0.15 us (1.210 -> 1.196
// ms against 0.25), adjoint at 0 (1.588 -> 1.562 ms), the defaults.  Timing only: results are
// identical for every delay.
#define PT_SWEEP_DELAY()                                                                            \
    if (a.sweep_delay > 0) {                                                                        \
        const unsigned long long d0_ = __builtin_amdgcn_s_memrealtime();                            \
        while (__builtin_amdgcn_s_memrealtime() - d0_ < (unsigned long long)a.sweep_delay)          \
            __builtin_amdgcn_s_sleep(1);                                                            \
    }

#define PT_PROF(ACC)                                                                                \
    if (prof) { const unsigned long long now_ = __builtin_amdgcn_s_memrealtime(); ACC += now_ - tm; tm = now_; }

// Re-materialise a wave-uniform value inside the time loop: stops the compiler from hoisting the
// per-row compares on it out of the loop as live 64-bit lane masks (which spill to VGPR lanes and
// cost v_readlane pairs in every step).
#define LAUNDER(x)                                                                                  \
    do {                                                                                            \
        x = __builtin_amdgcn_readfirstlane(x);   /* uniform by construction: never a VGPR->SGPR copy */ \
        asm volatile("" : "+s"(x));                                                                 \
    } while (0)

struct FwdPtArgs {
    TBGeo g;
    const float *coeffs;                 // alpha, temp1, temp2 at 0, 1, 2 x cstride; beta at 4
    const float *wav;                    // [nt] fp32 wavelet
    float *hist;                         // history base (slot j = P_{j-1}) or nullptr (no-grad)
    float *seis;
    unsigned long long *gran;
    unsigned *status;
    unsigned long long *prof;            // nullable: [0] hand-off, [1] steps, [2] publish (10 ns ticks), [3] waves
    int nt;
    int xcd_mode;                        // 1: XCD-local slices (pt_assign), 0: all hand-offs write-through
    int sweep_delay;                     // s_memrealtime ticks (10 ns) between an epoch's publish and its first sweep pass
};

// One forward step P_{n+1} = temp1 P_n - temp2 P_{n-1} + alpha N(P_n) (+ source), pde.py:79-81, on
// packed fp32: a wave's 8 rows are held as 4 row PAIRS {r, r+4} (float2 = one VGPR pair), so every
// add / mul of the stencil is one v_pk_*_f32 for two rows (IEEE-identical to the scalar ops, same
// operation order per row).  With this pairing the vertical neighbours of pair i are pairs i-1 /
// i+1 / i-2 / i+2 except at the slab ends, where four pairs are assembled from the halo rows.  The
// horizontal taps stay per-row DPP lane shifts (DPP has no packed form).
// (one descriptor per epoch, HFe = slot n0 + 2, and the step's slot as the scalar offset: no
// per-step 64-bit address arithmetic; the lanes' offsets stay OOB for cells the wave does not own)
#define FWD_HIST(V, N)                                                                              \
    {                                                                                               \
        const int so_ = ((N) - n0) * L4;                                                            \
        _Pragma("unroll") for (int r = 0; r < R; ++r)                                               \
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(PT_AT(V, r)), HFe, hv[r], so_, CP_NT); \
    }
// the receiver row's values of the epoch's steps n0 .. n0+T-1 (after the hand-off sweep): one buffer
// store per recorded step (lanes without a receiver at an OOB offset, the record row as the scalar
// offset), the per-column receiver lists only where a column has several
#define FWD_RECORD                                                                                  \
    {                                                                                               \
        int rrw_ = rrow;                                                                            \
        LAUNDER(rrw_);                                                                              \
        if (rrw_ >= 0) {                                                                            \
            _Pragma("unroll") for (int t = 0; t < T; ++t) {                                         \
                const int n = n0 + t;                                                               \
                const int ri_ = n < a.nt ? rec_index(n, g.st) : -1;                                 \
                if (ri_ >= 0) {                                                                     \
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(rv[t]), SKR, vrec, ri_ * ng4, 0); \
                    unsigned rm_ = rmulti;                                                          \
                    LAUNDER(rm_);                                                                   \
                    if (rm_ && rec) {                        /* several receivers in one column */  \
                        float *SK = a.seis + ((size_t)bs * g.nrec + ri_) * g.ng;                    \
                        for (int j = rs + 1; j < re; ++j) SK[g.rcv_list[j]] = rv[t];                \
                    }                                                                               \
                }                                                                                   \
            }                                                                                       \
        }                                                                                           \
    }

// Row r of a row-pair array.  Stacked pairs {i, i+RP} (PT_MIR false: the exact-order adjoint) or
// mirrored pairs {i, R-1-i} (PT_MIR true: the barrier-free kernels).  In the mirrored form the four
// boundary rows 0, 1, R-2, R-1 are pairs 0 and 1 alone, so a step can finish (and publish) them
// before its interior pairs; the vertical neighbours of pair i are still pairs i-1 / i+1 / i-2 /
// i+2 (the .y half runs the other way, and the stencil's sums are symmetric), except at the slab
// ends (halo rows) and in the middle, where a pair meets itself swapped.
template <int RP, bool M>
__device__ constexpr int pt_pair(int r) { return M ? (r < RP ? r : 2 * RP - 1 - r) : r % RP; }
template <int RP, bool M>
__device__ constexpr int pt_half(int r) { return M ? (r < RP ? 0 : 1) : r / RP; }
#define PT_AT(V, r) V[pt_pair<RP, PT_MIR>(r)][pt_half<RP, PT_MIR>(r)]
__device__ __forceinline__ f32x2 swp(f32x2 v) { return f32x2{v.y, v.x}; }
// vertical neighbours (rows -1, +1, -2, +2) of mirrored pair i of X; E1 = rows {-1, R}, E2 = {-2, R+1}
#define MIR_VERT(X, i, m1, p1, m2, p2)                                                              \
    const f32x2 m1 = (i) >= 1 ? X[(i) - 1] : E1;                                                    \
    const f32x2 p1 = (i) <= RP - 2 ? X[(i) + 1] : swp(X[RP - 1]);                                   \
    const f32x2 m2 = (i) >= 2 ? X[(i) - 2] : ((i) == 1 ? E1 : E2);                                  \
    const f32x2 p2 = (i) <= RP - 3 ? X[(i) + 2] : ((i) == RP - 2 ? swp(X[RP - 1]) : swp(X[RP - 2]));

// Barrier-free forward step: the halo-free work of every pair (DPP shifts, time
// terms) first, then the wait for the neighbours' boundary rows, the two boundary pairs, their
// publication for the next step, and the interior pairs after it.  Per row the operations and
// their order are the reference's (bit-exact).
#define FWD_PAIRS_NB(CUR, PRV, LO, HI)                                                                        \
    {                                                                                               \
        _Pragma("unroll") for (int i = (LO); i < (HI); ++i) {                                        \
            MIR_VERT(CUR, i, m1, p1, m2, p2)                                                        \
            f32x2 s1 = m1 + p1; s1 = s1 + xl1[i]; s1 = s1 + xr1[i];                                 \
            const f32x2 la = kC2 * s1;                                                              \
            f32x2 s2 = m2 + p2;                        /* x -+ 2 taps: fused v_add_f32_dpp */       \
            s2.x = s2.x + dpp_shr1(xl1[i].x); s2.y = s2.y + dpp_shr1(xl1[i].y);                     \
            s2.x = s2.x + dpp_shl1(xr1[i].x); s2.y = s2.y + dpp_shl1(xr1[i].y);                     \
            const f32x2 l2 = kC3 * s2; const f32x2 lap = la + l2;                                   \
            const f32x2 a3 = A[i] * lap;                                                            \
            PRV[i] = tt[i] + a3;                                                                    \
        }                                                                                           \
        unsigned sm0_ = (HI) > (LO) ? smask : 0u;                                                  \
        LAUNDER(sm0_);                               /* scalar branch; nothing of it hoisted */     \
        if (sm0_) {                                  /* pde.py:80-81 (uniform: source row waves) */ \
            float wt_ = wv[t];                                                                      \
            asm volatile("" : "+s"(wt_));                                                           \
            const float add = scol ? bsrc * wt_ : -0.0f;                                            \
            unsigned one_ = s1row;                                                                  \
            LAUNDER(one_);                                                                          \
            if (one_) {                                                                             \
                const f32x2 av = shalf ? f32x2{-0.0f, add} : f32x2{add, -0.0f};                     \
                int sp_ = spair;                                                                    \
                LAUNDER(sp_);                                                                       \
                _Pragma("unroll") for (int i = (LO); i < (HI); ++i)                                  \
                    if (i == sp_) PRV[i] = PRV[i] + av;                                             \
            } else {                                                                                \
                unsigned sm_ = smask;                                                               \
                LAUNDER(sm_);                                                                       \
                _Pragma("unroll") for (int r = 0; r < R; ++r)                                       \
                    if (pt_pair<RP, PT_MIR>(r) >= (LO) && pt_pair<RP, PT_MIR>(r) < (HI) && ((sm_ >> r) & 1u)) \
                        PT_AT(PRV, r) = PT_AT(PRV, r) + add;                                        \
            }                                                                                       \
        }                                                                                           \
    }
#define FWD_STEP_NB(CUR, PRV)                                                                       \
    {                                                                                               \
        u32x2 f_;                                                                                   \
        f32x2 E1, E2;                                                                               \
        xm_load<NW>(xm, n & 1, w, lane, f_, E1, E2);                                                \
        f32x2 xl1[RP], xr1[RP], tt[RP];                                                             \
        _Pragma("unroll") for (int i = 0; i < RP; ++i) {                                             \
            const f32x2 c = CUR[i];                                                                 \
            xl1[i] = f32x2{dpp_shr1(c.x), dpp_shr1(c.y)};                                           \
            xr1[i] = f32x2{dpp_shl1(c.x), dpp_shl1(c.y)};                                           \
            f32x2 a1 = C1[i] * c; const f32x2 a2 = C2v[i] * PRV[i]; a1 = a1 - a2;                   \
            tt[i] = a1;                                                                             \
            asm volatile("" : "+v"(tt[i]));          /* computed here, not sunk past the wait */    \
        }                                                                                           \
        xm_wait<NW>(xm, n & 1, w, lane, (unsigned)n + 1u, f_, E1, E2, a.status, live);              \
        FWD_PAIRS_NB(CUR, PRV, 0, 2)                                                                          \
        if (t + 1 < T) xm_put<NW>(xm, (n + 1) & 1, w, lane, (unsigned)n + 2u, PRV[0], PRV[1]);      \
        __builtin_amdgcn_s_setprio(PT_PRIO_BODY);                                                   \
        FWD_PAIRS_NB(CUR, PRV, 2, RP)                                                                         \
        if (a.hist && (t + 1 < T || e + 1 == nep)) FWD_HIST(PRV, n)                                 \
        int rr_ = rrow;                                                                             \
        LAUNDER(rr_);                                                                               \
        if (rr_ >= 0) {                              /* receiver row: value kept, stored per epoch */ \
            int rp_ = rpair;                                                                        \
            LAUNDER(rp_);                                                                           \
            f32x2 v_ = PRV[0];                                                                      \
            _Pragma("unroll") for (int i = 1; i < RP; ++i) if (i == rp_) v_ = PRV[i];                \
            rv[t] = rhalf ? v_.y : v_.x;                                                            \
        }                                                                                           \
    }

template <int T, int NW, int RW, bool PROF>
__global__ __launch_bounds__(64 * NW) void k_fwd_pt(FwdPtArgs a)
{
    unsigned long long *const prof = PROF ? a.prof : nullptr;   // phase counters: profiled build only
    constexpr bool PT_MIR = true;                         // mirrored pairs (barrier-free exchange:
                                                          // 1.364 -> 1.287 ms at configs[1])
    constexpr bool PT_PRIO = true;                        // wave priorities (PT_PRIO_*)
    __shared__ XmBox<NW> xm;                              // the waves' inboxes (xm_*)
    const TBGeo &g = a.g;
    PT_REGION_INIT(NW, RW)
    const float *AL = a.coeffs + (size_t)b * g.slice;
    f32x2 A[RP], C1[RP], C2v[RP], P0[RP], P1[RP];         // row pairs {r, r+RP}: PT_AT(X, r)
    const f32x2 kC2 = {C2, C2}, kC3 = {C3, C3};
    unsigned smask = 0;
    int rrow = -1;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int gz = wrap_row(uz0 + r, g.Hp);
        const int o = gz * g.ld + gx;
        PT_AT(A, r) = AL[o]; PT_AT(C1, r) = AL[g.cstride + o]; PT_AT(C2v, r) = AL[2 * g.cstride + o];
        PT_AT(P0, r) = 0.0f; PT_AT(P1, r) = 0.0f;         // P_{-1} = P_0 = 0 (pde.py:74-75)
        if (gz == g.isz) smask |= 1u << r;
        if (gz == g.igz && ((rin >> r) & 1u)) rrow = r;
    }
    smask = __builtin_amdgcn_readfirstlane(smask);        // wave-uniform (row-only): scalar branches,
    rrow = __builtin_amdgcn_readfirstlane(rrow);          // no per-lane masks held across the loop
    const int isx = g.isx[s];
    const bool scol = gx == isx;
    const float bsrc = (smask != 0) ? AL[4 * g.cstride + (size_t)g.isz * g.ld + isx] : 0.0f;

    int rs = 0, re = 0, rcv0 = -1;
    if (rrow >= 0) {
        rs = g.rcv_start[gx]; re = g.rcv_start[gx + 1];
        rcv0 = rs < re ? g.rcv_list[rs] : -1;             // the (usually only) receiver of this column
    }
    const bool rec = rrow >= 0 && xin && rcv0 >= 0;
    const unsigned rmulti = __any(re - rs > 1);           // wave-uniform: a column with several receivers
    const __amdgpu_buffer_rsrc_t SKR = rsrc_of(a.seis + (size_t)bs * g.nrec * g.ng);   // FWD_RECORD
    const int vrec = rec ? rcv0 * 4 : OOB, ng4 = g.ng * 4;
    // source / receiver rows as (row pair, half): the step touches one pair, not all eight rows
    const unsigned s1row = smask != 0 && (smask & (smask - 1u)) == 0;   // one source row in the slab
    const int sr1 = smask ? __builtin_ctz(smask) : 0;
    // wave-uniform by construction; readfirstlane makes that visible to the compiler (LAUNDER "+s")
    const int spair = __builtin_amdgcn_readfirstlane(PT_MIR ? (sr1 < RP ? sr1 : R - 1 - sr1) : sr1 % RP);
    const int rpair = __builtin_amdgcn_readfirstlane(rrow < 0 ? 0 : PT_MIR ? (rrow < RP ? rrow : R - 1 - rrow) : rrow % RP);
    const bool shalf = sr1 >= RP, rhalf = rrow >= RP;     // the half is r >= RP in both pairings
    float rv[T];
#pragma unroll
    for (int t = 0; t < T; ++t) rv[t] = 0.0f;
    const size_t L = g.level;
    const int L4 = (int)(L * 4);                          // bytes per history slot (< 2 GB: resident surveys)
    int hv[R];                                            // history store offset of (row, lane), OOB if not own
#pragma unroll
    for (int r = 0; r < R; ++r) hv[r] = (((rin >> r) & 1u) && xin) ? (PT_ROFS(r) + gx) * 4 : OOB;
    const int nep = (a.nt + T - 1) / T;
    bool live = true;
    unsigned long long tsw = 0, tst = 0, tpb = 0, tm = prof ? __builtin_amdgcn_s_memrealtime() : 0;
    unsigned long long tfp = 0, npass = 0;                // profile: first-pass latency, sweep passes
    // The next epoch's wavelet samples (FWD_ISSUE) are scalar loads issued right after the publish: the
    // source row's first step no longer waits for them behind the deferred history stores.
    float wv[T];
#pragma unroll
    for (int t = 0; t < T; ++t) wv[t] = wav_s(a.wav, min(t, a.nt - 1));
    __builtin_amdgcn_s_waitcnt(0x0F70);                   // vmcnt(0)
#define FWD_ISSUE _Pragma("unroll") for (int t = 0; t < T; ++t) wv[t] = wav_s(a.wav, min(n0 + T + t, a.nt - 1));
    xm_init<NW>(xm, w, lane);                             // no flag matches a tag until written
    __syncthreads();
    xm_put<NW>(xm, 0, w, lane, 1u, f32x2{0.0f, 0.0f}, f32x2{0.0f, 0.0f});   // P_0 = 0, step 0's tag
#define FWD_STEP_SEL FWD_STEP_NB
    for (int e = 0; e < nep; ++e) {
        const int n0 = e * T;
        const __amdgpu_buffer_rsrc_t HFe = rsrc_of(a.hist + (size_t)(n0 + 2) * L + so);   // FWD_HIST
        PT_PROF(tsw)
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const int n = n0 + t;
            if (n >= a.nt) break;
            if (t & 1) FWD_STEP_SEL(P0, P1)
            else FWD_STEP_SEL(P1, P0)
        }
        if (T & 1) {   // keep "P1 = newest" at every epoch boundary
#pragma unroll
            for (int i = 0; i < RP; ++i) { const f32x2 tmp = P0[i]; P0[i] = P1[i]; P1[i] = tmp; }
        }
        PT_PROF(tst)
        if (e + 1 < nep) {
            const unsigned tag = (unsigned)(e + 1);
            const __amdgpu_buffer_rsrc_t GR = rsrc_of(a.gran + (size_t)(2 * ((e + 1) & 1)) * L + 2 * so);
            PT_PUBLISH(GR, tag, P0, P1)
            PT_PROF(tpb)
            FWD_ISSUE                                     // scalar loads (wav_s): their latency hides in the
                                                          // delay and the sweep, and no vector op waits on them
            PT_SWEEP_DELAY()
            PT_SWEEP(GR, tag, P0, P1, R)
            if (a.hist) FWD_HIST(P1, n0 + T - 1)          // the epoch's last step (own cells: the sweep
                                                          // reloads halo cells only)
            // the next step's boundary rows, with the halo cells the sweep reloaded
            xm_put<NW>(xm, (n0 + T) & 1, w, lane, (unsigned)(n0 + T) + 1u, P1[0], P1[1]);
        }
        FWD_RECORD
    }
#undef FWD_STEP_SEL
#undef FWD_ISSUE
    PT_PROF(tsw)
    if (prof && lane == 0) {
        atomicAdd(prof + 0, tsw); atomicAdd(prof + 1, tst); atomicAdd(prof + 2, tpb); atomicAdd(prof + 3, 1ull);
        atomicAdd(prof + 4, tfp); atomicAdd(prof + 5, npass);
        if (blockIdx.x < PROF_WAVES / 16) {
            unsigned long long *raw = prof + PROF_RAW + ((size_t)blockIdx.x * 16 + w) * 3;   // per wave
            raw[0] = tsw; raw[1] = tst; raw[2] = tpb;
        }
    }
}

#undef FWD_HIST
#undef FWD_RECORD

// The adjoint keeps the forward's row-pair packing (PT_AT(V, r) = V[r % RP][r / RP]): every add /
// mul / fma of the step and of the gradient is one v_pk_*_f32 for two rows.

struct AdjPtArgs {
    TBGeo g;
    const float *coeffs;                 // alpha, temp1, temp2, kappa at 0..3 x cstride
    const float *wav;
    const float *hist;                   // slot k = P_{k-1}
    const float *dseis;
    float *gA;                           // [B][ns][Hp][ld]
    double *gk_part;                     // [B*ns][nblk]
    float *gbeta;                        // [B*ns]
    unsigned long long *gran;
    unsigned *status;
    unsigned long long *prof;            // nullable, as FwdPtArgs
    int nt, nblk;
    int xcd_mode;
    int sweep_delay;                     // as FwdPtArgs
};

__device__ __forceinline__ float bload_nt(__amdgpu_buffer_rsrc_t r, int voff, int soff)
{
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, CP_NT));
}

// P_{k-1}, rows uz0-2 .. uz0+9 of one step: slab rows 0..7 as row pairs PC[i] = {i, i+4}, the
// stencil's halo rows as PH = {-2, -1, 8, 9}.  HR = the epoch's history descriptor, SOFF = the
// step's slot offset inside it (bytes): one 64-bit descriptor per epoch, not per step.
#define ADJ_PLOAD(PC, PH, HR, SOFF)                                                                 \
    {                                                                                               \
        const int so_ = (SOFF);                                                                     \
        _Pragma("unroll") for (int i = 0; i < RP; ++i) {                                             \
            PC[i].x = bload_nt(HR, pv[i + 2], so_);                                                 \
            PC[i].y = bload_nt(HR, pv[i + 6], so_);                                                 \
        }                                                                                           \
        PH[0] = bload_nt(HR, pv[0], so_); PH[1] = bload_nt(HR, pv[1], so_);                         \
        PH[2] = bload_nt(HR, pv[10], so_); PH[3] = bload_nt(HR, pv[11], so_);                       \
    }

// vertical neighbours of row pair i in a row-pair field X whose four outer rows are in
// eU1 = {-1, RP-1}, eU2 = {-2, RP-2}, eD1 = {RP, R}, eD2 = {RP+1, R+1}
#define PAIR_VERT(X, i, m1, p1, m2, p2)                                                             \
    const f32x2 m1 = (i) >= 1 ? X[(i) - 1] : eU1;                                                   \
    const f32x2 p1 = (i) <= RP - 2 ? X[(i) + 1] : eD1;                                              \
    const f32x2 m2 = (i) >= 2 ? X[(i) - 2] : ((i) == 1 ? eU1 : eU2);                                \
    const f32x2 p2 = (i) <= RP - 3 ? X[(i) + 2] : ((i) == RP - 2 ? eD1 : eD2);

// gradient accumulation of one step (interior rows are the ones stored; every row of a wave that
// has interior rows is computed: no per-row branch).  CU = L_{k+1}, LN = L_k, P / PH = P_{k-1}.
//   gA_s += L_k (2c1 P + c2 S1(P) + c3 S2(P)),  GK += P (L_{k+1} - L_k)  (x K once at the end),
//   gbeta[s] += L_k(src) w[k-1]
#define ADJ_GRAD(CU, LN, P, PH, WK)                                                                 \
    if (grad) {                                                                                     \
        const f32x2 eU1 = {PH[1], P[RP - 1].x}, eU2 = {PH[0], P[RP - 2].x};                         \
        const f32x2 eD1 = {P[0].y, PH[2]}, eD2 = {P[1].y, PH[3]};                                   \
        _Pragma("unroll") for (int i = 0; i < RP; ++i) {                                             \
            PAIR_VERT(P, i, m1, p1, m2, p2)                                                         \
            const f32x2 c = P[i];                                                                   \
            const f32x2 xl1 = {dpp_shr1(c.x), dpp_shr1(c.y)}, xr1 = {dpp_shl1(c.x), dpp_shl1(c.y)}; \
            f32x2 s1 = m1 + p1; s1 = s1 + xl1; s1 = s1 + xr1;                                       \
            f32x2 s2 = m2 + p2;                        /* x -+ 2 taps: fused v_add_f32_dpp */       \
            s2.x = s2.x + dpp_shr1(xl1.x); s2.y = s2.y + dpp_shr1(xl1.y);                           \
            s2.x = s2.x + dpp_shl1(xr1.x); s2.y = s2.y + dpp_shl1(xr1.y);                           \
            const f32x2 l = LN[i];                                                                  \
            f32x2 lap = kC2 * s1; const f32x2 lq = kC3 * s2; lap = lap + lq;                        \
            f32x2 d = kC1X2 * c; d = d + lap;                                                       \
            const f32x2 cc = l * d;                                                                 \
            GA[i] = GA[i] + cc;                                                                     \
            f32x2 kk = KP[i] * c; const f32x2 dl = CU[i] - l; kk = kk * dl;   /* fp32 term */       \
            if (xin) {                                                       /* fp64 sum */        \
                if ((rin >> i) & 1u) ksum += (double)kk.x;                                          \
                if ((rin >> (i + RP)) & 1u) ksum += (double)kk.y;                                   \
            }                                                                                       \
        }                                                                                           \
        if (srow >= 0) {                             /* gbeta: the source cell's lane only */      \
            int sr_ = srow;                                                                         \
            LAUNDER(sr_);                                                                           \
            float ls_ = 0.0f;                                                                       \
            _Pragma("unroll") for (int r = 0; r < R; ++r) if (r == sr_) ls_ = PT_AT(LN, r);         \
            const float gb = scol ? ls_ * (WK) : -0.0f;                                             \
            gbacc = gbacc + gb;                                                                     \
        }                                                                                           \
    }

// one adjoint step k: CUR = L_{k+1}, PRV = L_{k+2} -> L_k; P / PH = P_{k-1}; the
// next step's P_{k-2} is prefetched into PN / PHN.  The gradient of the epoch's last step is
// deferred past the publish (see k_adj_pt).
#define ADJ_STEP(CUR, PRV, P, PH, PN, PHN)                                                          \
    {                                                                                               \
        if (t + 1 < T) ADJ_PLOAD(PN, PHN, HRe, (T - 2 - t) * L4)                                    \
        const float dcur = dv[t];                                                                   \
        f32x2 q[RP];                                                                                \
        _Pragma("unroll") for (int i = 0; i < RP; ++i) q[i] = A[i] * CUR[i];                         \
        const Halo4 h4 = exchange_nw<NW>(xch, j & 1, w, lane, q[0].x, q[1].x, q[RP - 2].y, q[RP - 1].y); \
        const f32x2 eU1 = {h4.u1, q[RP - 1].x}, eU2 = {h4.u2, q[RP - 2].x};                         \
        const f32x2 eD1 = {q[0].y, h4.d1}, eD2 = {q[1].y, h4.d2};                                   \
        _Pragma("unroll") for (int i = 0; i < RP; ++i) {                                             \
            PAIR_VERT(q, i, m1, p1, m2, p2)                                                         \
            const f32x2 c = q[i];                                                                   \
            const f32x2 xl1 = {dpp_shr1(c.x), dpp_shr1(c.y)}, xr1 = {dpp_shl1(c.x), dpp_shl1(c.y)}; \
            f32x2 n1 = m1 + p1; n1 = n1 + xl1; n1 = n1 + xr1;                                       \
            f32x2 n2 = m2 + p2;                        /* x -+ 2 taps: fused v_add_f32_dpp */       \
            n2.x = n2.x + dpp_shr1(xl1.x); n2.y = n2.y + dpp_shr1(xl1.y);                           \
            n2.x = n2.x + dpp_shl1(xr1.x); n2.y = n2.y + dpp_shl1(xr1.y);                           \
            f32x2 nb = kC2 * n1; const f32x2 nb2 = kC3 * n2; nb = nb + nb2;                         \
            f32x2 l = T1v[i] * CUR[i]; const f32x2 l2 = T2v[i] * PRV[i]; l = l - l2; l = l + nb;     \
            PRV[i] = l;                                                                             \
        }                                                                                           \
        if (rrow >= 0 && rec_index(k - 1, g.st) >= 0) {   /* uniform: the receiver row's wave */    \
            int rr_ = rrow;                                                                         \
            LAUNDER(rr_);                                                                           \
            _Pragma("unroll") for (int r = 0; r < R; ++r)                                           \
                if (r == rr_) PT_AT(PRV, r) = PT_AT(PRV, r) + dcur;   /* -0 off the receivers */     \
        }                                                                                           \
        if (t + 1 < T || last) ADJ_GRAD(CUR, PRV, P, PH, wv[t])                                     \
    }

// Adjoint, persistent, in the oracle's exact fp32 operation order (rdq_fwi_set_variant flag 2: the
// bitwise tests; the default build is k_adj_pr below).  Per step k = nt..1:
//   L_k = T1 L_{k+1} - T2 L_{k+2} + (c2 N1(A L_{k+1}) + c3 N2(A L_{k+1})) [+ R^T dseis[k-1]]
//   gA_s += L_k (2c1 P_{k-1} + c2 S1(P_{k-1}) + c3 S2(P_{k-1})),  gk += (K P_{k-1})(L_{k+1} - L_k),
//   gbeta[s] += L_k(src) w[k-1]        (interior cells; accumulators in registers for all nt steps)
// P_{k-1} comes from the history: each wave loads its rows +-2 one step ahead into alternating
// register arrays and needs no LDS exchange for it.  Per epoch of T steps: steps, publish of the
// border, then the LAST step's gradient (it needs no neighbour data: the interior L_k, L_{k+1} and
// the wave's own history rows), and only then the hand-off sweep — the gradient's VALU work fills
// the time the neighbours' granules take to arrive.
template <int T, int NW, bool PROF>
__global__ __launch_bounds__(64 * NW) void k_adj_pt(AdjPtArgs a)
{
    unsigned long long *const prof = PROF ? a.prof : nullptr;   // phase counters: profiled build only
    constexpr bool PT_MIR = false;                        // stacked pairs {i, i+4} (ADJ_PLOAD / ADJ_GRAD)
    constexpr bool PT_PRIO = false;                       // (barrier-synchronised steps: PT_PRIO_*)
    __shared__ float xch[2][NW][4][64];
    __shared__ double red[64 * NW];
    const TBGeo &g = a.g;
    PT_REGION_INIT(NW, TB_R)
    const float *AL = a.coeffs + (size_t)b * g.slice;
    f32x2 A[RP], T1v[RP], T2v[RP], KP[RP], L0[RP], L1[RP], GA[RP];
    const f32x2 kC2 = {C2, C2}, kC3 = {C3, C3}, kC1X2 = {C1X2, C1X2};
    int srow = -1, rrow = -1;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int gz = wrap_row(uz0 + r, g.Hp);
        const int o = gz * g.ld + gx;
        PT_AT(A, r) = AL[o]; PT_AT(T1v, r) = AL[g.cstride + o]; PT_AT(T2v, r) = AL[2 * g.cstride + o];
        PT_AT(KP, r) = AL[3 * g.cstride + o];
        PT_AT(L0, r) = 0.0f; PT_AT(L1, r) = 0.0f;         // L_{nt+1} = L_{nt+2} = 0
        PT_AT(GA, r) = 0.0f;
        if (gz == g.isz && ((rin >> r) & 1u)) srow = r;
        if (gz == g.igz) rrow = r;
    }
    const bool scol = xin && gx == g.isx[s];
    // residual of this lane's column: one receiver's dseis, or several receivers' folded sum
    const int rcv0 = rrow >= 0 ? g.rlane[gx] : -1;
    const float *DSb = a.dseis + (size_t)bs * g.nrec * g.dstride;
    const __amdgpu_buffer_rsrc_t DSR = rsrc_of(DSb);
    // dseis[k-1] of this lane's receiver; -0 (x + -0 == x bitwise) where there is none.  An
    // unconditional buffer load (OOB offset: no memory access) keeps every wave's vmcnt count equal.
#define DLOAD(KK)                                                                                   \
    ({                                                                                              \
        const int ri_ = (KK) >= 1 ? rec_index((KK) - 1, g.st) : -1;                                 \
        const bool ok_ = rcv0 >= 0 && ri_ >= 0;                                                     \
        const float v_ = bload(DSR, ok_ ? (ri_ * g.dstride + rcv0) * 4 : OOB, 0);                   \
        ok_ ? v_ : -0.0f;                                                                           \
    })
    const bool grad = rin != 0;                           // uniform: this wave has interior rows
    double ksum = 0.0;
    float gbacc = 0.0f;
    const size_t L = g.level;
    const int L4 = (int)(L * 4);                          // bytes per history slot (< 2 GB: resident surveys)
    f32x2 PA[RP], PB[RP];
    float PHA[4], PHB[4];
    int pv[12];                                           // P row (uz0 - 2 + i) offset of this lane
#pragma unroll
    for (int i = 0; i < 12; ++i) pv[i] = grad ? (wrap_row(uz0 + i - 2, g.Hp) * g.ld + gx) * 4 : OOB;
    // history descriptor of the epoch whose first step is KN: slots KN - T + 1 .. KN (step t of the
    // epoch reads slot KN - t at byte offset (T - 1 - t) * L4)
#define HIST_RSRC(KN) rsrc_of(a.hist + (ptrdiff_t)((KN) - (T - 1)) * (ptrdiff_t)L + (ptrdiff_t)so)
    // Per-epoch inputs (the first step's history slice P, the receiver residuals dseis[k-1] and the
    // wavelet w[k-1] of the epoch's T steps) are issued right behind the hand-off loads of the
    // previous epoch's sweep (ADJ_ISSUE), so the sweep does not wait for this HBM traffic; inside an
    // epoch a step waits only for its own P (prefetched one step ahead).
    float wv[T], dv[T];
    {
        const __amdgpu_buffer_rsrc_t H0 = HIST_RSRC(a.nt);
        ADJ_PLOAD(PA, PHA, H0, (T - 1) * L4)
    }
#pragma unroll
    for (int t = 0; t < T; ++t) {
        wv[t] = a.wav[max(a.nt - t - 1, 0)];
        dv[t] = DLOAD(a.nt - t);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);                   // vmcnt(0)
#define ADJ_ISSUE                                                                                   \
    {                                                                                               \
        const __amdgpu_buffer_rsrc_t HN = HIST_RSRC(kn);                                            \
        ADJ_PLOAD(PA, PHA, HN, (T - 1) * L4)                                                        \
        _Pragma("unroll") for (int t = 0; t < T; ++t) {                                             \
            wv[t] = a.wav[max(kn - t - 1, 0)];                                                      \
            dv[t] = DLOAD(kn - t);                                                                  \
        }                                                                                           \
    }
    const int nep = (a.nt + T - 1) / T;
    bool live = true;
    unsigned long long tsw = 0, tst = 0, tpb = 0, tm = prof ? __builtin_amdgcn_s_memrealtime() : 0;
    unsigned long long tfp = 0, npass = 0;                // profile: first-pass latency, sweep passes
    for (int e = 0; e < nep; ++e) {
        const int ke = a.nt - e * T;                      // first step k of this epoch
        const bool last = e + 1 == nep;
        const __amdgpu_buffer_rsrc_t HRe = HIST_RSRC(ke);
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const int j = e * T + t;
            if (j >= a.nt) break;
            const int k = ke - t;
            if (t & 1) ADJ_STEP(L0, L1, PB, PHB, PA, PHA)
            else ADJ_STEP(L1, L0, PA, PHA, PB, PHB)
        }
        if (T & 1) {   // keep "L1 = newest, PB = the last step's P, PA = free" at every epoch boundary
#pragma unroll
            for (int i = 0; i < RP; ++i) {
                const f32x2 tl = L0[i]; L0[i] = L1[i]; L1[i] = tl;
                const f32x2 tp = PA[i]; PA[i] = PB[i]; PB[i] = tp;
                const float th = PHA[i]; PHA[i] = PHB[i]; PHB[i] = th;
            }
        }
        PT_PROF(tst)
        if (!last) {
            const unsigned tag = (unsigned)(e + 1);
            const __amdgpu_buffer_rsrc_t GR = rsrc_of(a.gran + (size_t)(2 * ((e + 1) & 1)) * L + 2 * so);
            PT_PUBLISH(GR, tag, L0, L1)
            ADJ_GRAD(L0, L1, PB, PHB, wv[T - 1])          // the deferred last step (no neighbour data)
            const int kn = ke - T;                        // first step k of the next epoch
            PT_PROF(tpb)
            PT_SWEEP_DELAY()
            PT_SWEEP(GR, tag, L0, L1, PT_ADJ_SG)
            ADJ_ISSUE
            PT_PROF(tsw)
        }
    }
#undef DLOAD
#undef ADJ_ISSUE
#undef HIST_RSRC
    if (prof && lane == 0) {
        atomicAdd(prof + 0, tsw); atomicAdd(prof + 1, tst); atomicAdd(prof + 2, tpb); atomicAdd(prof + 3, 1ull);
        atomicAdd(prof + 4, tfp); atomicAdd(prof + 5, npass);
        if (blockIdx.x < PROF_WAVES / 16) {
            unsigned long long *raw = prof + PROF_RAW + ((size_t)blockIdx.x * 16 + w) * 3;   // per wave
            raw[0] = tsw; raw[1] = tst; raw[2] = tpb;
        }
    }
    if (xin) {
#pragma unroll
        for (int r = 0; r < R; ++r)
            if ((rin >> r) & 1u) a.gA[so + (size_t)PT_ROFS(r) + gx] = PT_AT(GA, r);
    }
    if (srow >= 0 && scol) a.gbeta[bs] = gbacc;
    // deterministic workgroup reduction of the sponge-coefficient partial sum
    const int tid = threadIdx.x;
    red[tid] = ksum;
    __syncthreads();
    for (int w2 = 512; w2 > 0; w2 >>= 1) {
        if (tid < w2 && tid + w2 < 64 * NW) red[tid] += red[tid + w2];
        __syncthreads();
    }
    if (tid == 0) a.gk_part[(size_t)bs * a.nblk + tile] = red[0];
}
// ---- FMA build of the persistent adjoint: the gradient from the history's time recurrence.
// The forward's own update P_k = T1 P_{k-1} - T2 P_{k-2} + A lap'(P_{k-1}) (+ beta w[k-1] at the
// source cell, pde.py:79-81) gives the stencil term the gradient needs without a stencil:
//   lap'(P_{k-1}) = (P_k - T1 P_{k-1} + T2 P_{k-2} - src) / A,   d = 2c1 P_{k-1} + lap'(P_{k-1})
// so a step's gradient is 7 packed ops per row pair (no DPP, no P halo rows, 8 history rows per
// wave and step instead of 12).  The history values are the forward's own, so the identity holds
// up to the rounding of P_k's last add (fp32 tolerance, like the FMA contraction of the step).
// The window lives in four row-pair buffers Q0..Q3 that rotate by one per step (step t of an
// epoch: P_k, P_{k-1}, P_{k-2} = Q[t], Q[t+1], Q[t+2] mod 4, prefetch into Q[t+3]): no copies for
// T = 4; other depths restore the order once per epoch.

#define ADJR_LOAD(PD, HR, SOFF)                                                                     \
    {                                                                                               \
        const int so_ = (SOFF);                                                                     \
        _Pragma("unroll") for (int i = 0; i < RP; ++i) {                                             \
            PD[i].x = bload_nt(HR, pr[i], so_);                                                     \
            PD[i].y = bload_nt(HR, pr[PT_MIR ? R - 1 - i : i + RP], so_);                           \
        }                                                                                           \
    }

// gradient of step k (CU = L_{k+1}, LN = L_k; wavelet sample WK = w[k-1]; window P0 = P_k,
// P1 = P_{k-1}, P2 = P_{k-2}): u = lap'(P_{k-1}) x A from the history (the forward's source add undone
// on the source row), d = 2c1 P_{k-1} + lap'(P_{k-1}), then the accumulations with L_k; the source
// row's two terms share one scalar branch.
#define ADJR_GRAD(CU, LN, WK, P0, P1, P2)                                                           \
    if (grad) {                                                                                     \
        f32x2 u[RP];                                                                                \
        _Pragma("unroll") for (int i = 0; i < RP; ++i) {                                             \
            u[i] = fma2(-T1v[i], P1[i], P0[i]);                                                     \
            u[i] = fma2(T2v[i], P2[i], u[i]);                                                       \
        }                                                                                           \
        int sg_ = srow;                              /* one scalar branch for both source terms */  \
        LAUNDER(sg_);                                                                               \
        if (sg_ >= 0) {                                                                             \
            int sp_ = spair;                                                                        \
            LAUNDER(sp_);                                                                           \
            const float sa_ = scol ? bsrc * (WK) : 0.0f;  /* the forward's source add, undone */    \
            const f32x2 sv_ = shalf ? f32x2{0.0f, sa_} : f32x2{sa_, 0.0f};                          \
            f32x2 lp_ = LN[0];                                                                      \
            _Pragma("unroll") for (int i = 0; i < RP; ++i) {                                         \
                if (i == sp_) u[i] = u[i] - sv_;                                                    \
                if (i > 0 && i == sp_) lp_ = LN[i];                                                 \
            }                                                                                       \
            const float ls_ = shalf ? lp_.y : lp_.x;                                                \
            const float gb = scol ? ls_ * (WK) : -0.0f;  /* gbeta: the source cell's lane only */   \
            gbacc = gbacc + gb;                                                                     \
        }                                                                                           \
        /* A d = A 2c1 P_{k-1} + u: the 1/A is applied once to the sum (gA = sum L A d / A) */     \
        _Pragma("unroll") for (int i = 0; i < RP; ++i) {                                             \
            const f32x2 dd = fma2(A[i], kC1X2 * P1[i], u[i]);                                       \
            GA[i] = fma2(LN[i], dd, GA[i]);                                                         \
            GK[i] = fma2(P1[i], CU[i] - LN[i], GK[i]);                                              \
        }                                                                                           \
    }

// one adjoint step k: CUR = L_{k+1}, PRV = L_{k+2} -> L_k; window P0 / P1 / P2 as ADJR_GRAD;
// history slot k-2 (the next step's P_{k-3}) prefetched into PN.  (Moving the gradient's history
// half between the barrier and the halo reads' use, as the forward does with its halo-free work,
// needs 8 more VGPRs than the 168 that 3 waves / SIMD allow: it spilled and ran 2.6x slower.)
#define ADJR_STEP(CUR, PRV, P0, P1, P2, PN)                                                         \
    {                                                                                               \
        if (grad && k >= 2) ADJR_LOAD(PN, HRe, (T - 1 - t) * L4)                                    \
        const float dcur = dv[t];                                                                   \
        f32x2 q[RP];                                                                                \
        _Pragma("unroll") for (int i = 0; i < RP; ++i) q[i] = A[i] * CUR[i];                         \
        const Halo4 h4 = exchange_nw<NW>(xch, j & 1, w, lane, q[0].x, q[1].x, q[RP - 2].y, q[RP - 1].y); \
        const f32x2 eU1 = {h4.u1, q[RP - 1].x}, eU2 = {h4.u2, q[RP - 2].x};                         \
        const f32x2 eD1 = {q[0].y, h4.d1}, eD2 = {q[1].y, h4.d2};                                   \
        _Pragma("unroll") for (int i = 0; i < RP; ++i) {                                             \
            PAIR_VERT(q, i, m1, p1, m2, p2)                                                         \
            const f32x2 c = q[i];                                                                   \
            const f32x2 xl1 = {dpp_shr1(c.x), dpp_shr1(c.y)}, xr1 = {dpp_shl1(c.x), dpp_shl1(c.y)}; \
            f32x2 n1 = m1 + p1; n1 = n1 + xl1; n1 = n1 + xr1;                                       \
            f32x2 n2 = m2 + p2;                        /* x -+ 2 taps: fused v_add_f32_dpp */       \
            n2.x = n2.x + dpp_shr1(xl1.x); n2.y = n2.y + dpp_shr1(xl1.y);                           \
            n2.x = n2.x + dpp_shl1(xr1.x); n2.y = n2.y + dpp_shl1(xr1.y);                           \
            const f32x2 nb = fma2(kC3, n2, kC2 * n1);                                               \
            PRV[i] = fma2(T1v[i], CUR[i], fma2(-T2v[i], PRV[i], nb));                               \
        }                                                                                           \
        if (rrow >= 0 && rec_index(k - 1, g.st) >= 0) {   /* uniform: the receiver row's wave */    \
            int rp_ = rpair;                                 /* one packed add on the row's pair */  \
            LAUNDER(rp_);                                                                           \
            const f32x2 dv_ = rhalf ? f32x2{-0.0f, dcur} : f32x2{dcur, -0.0f};   /* -0: no-op */     \
            _Pragma("unroll") for (int i = 0; i < RP; ++i) if (i == rp_) PRV[i] = PRV[i] + dv_;      \
        }                                                                                           \
        if (t + 1 < T || last) ADJR_GRAD(CUR, PRV, wv[t], P0, P1, P2)                               \
    }

// Barrier-free adjoint step (mirrored pairs, the forward's LDS mailbox xm_*): the wave waits
// only for its two neighbours' A L_{k+1} boundary rows, computes its two boundary pairs (receiver
// residual included), publishes their A L_k rows for the next step, then its interior pair.  Per row
// the operations and their order are ADJR_STEP's (m1 + p1 commutes: same bits).  (The gradient's
// history half ahead of the wait, as the forward's time terms, needs 6 more VGPRs: 84 B/lane scratch.)
#define ADJR_PAIRS_NB(CUR, PRV, LO, HI)                                                             \
    {                                                                                               \
        _Pragma("unroll") for (int i = (LO); i < (HI); ++i) {                                        \
            MIR_VERT(q, i, m1, p1, m2, p2)                                                          \
            const f32x2 c = q[i];                                                                   \
            const f32x2 xl1 = {dpp_shr1(c.x), dpp_shr1(c.y)}, xr1 = {dpp_shl1(c.x), dpp_shl1(c.y)}; \
            f32x2 n1 = m1 + p1; n1 = n1 + xl1; n1 = n1 + xr1;                                       \
            f32x2 n2 = m2 + p2;                        /* x -+ 2 taps: fused v_add_f32_dpp */       \
            n2.x = n2.x + dpp_shr1(xl1.x); n2.y = n2.y + dpp_shr1(xl1.y);                           \
            n2.x = n2.x + dpp_shl1(xr1.x); n2.y = n2.y + dpp_shl1(xr1.y);                           \
            const f32x2 nb = fma2(kC3, n2, kC2 * n1);                                               \
            PRV[i] = fma2(T1v[i], CUR[i], fma2(-T2v[i], PRV[i], nb));                               \
        }                                                                                           \
        int rr_ = (LO) == 0 ? rlo : rhi;             /* the receiver's pair is in this half */      \
        LAUNDER(rr_);                                                                               \
        if ((HI) > (LO) && rr_ && rec_index(k - 1, g.st) >= 0) {                                    \
            int rp_ = rpair;                                                                        \
            LAUNDER(rp_);                                                                           \
            const f32x2 dv_ = rhalf ? f32x2{-0.0f, dcur} : f32x2{dcur, -0.0f};   /* -0: no-op */     \
            _Pragma("unroll") for (int i = (LO); i < (HI); ++i) if (i == rp_) PRV[i] = PRV[i] + dv_; \
        }                                                                                           \
    }
#define ADJR_STEP_NB(CUR, PRV, P0, P1, P2, PN)                                                      \
    {                                                                                               \
        if (ldall || (grad && k >= 2)) ADJR_LOAD(PN, HRe, (T - 1 - t) * L4)                         \
        const float dcur = dv[t];                                                                   \
        u32x2 f_;                                                                                   \
        f32x2 E1, E2;                                                                               \
        xm_load<NW>(xm, j & 1, w, lane, f_, E1, E2);                                                \
        f32x2 q[RP];                                                                                \
        _Pragma("unroll") for (int i = 0; i < RP; ++i) q[i] = A[i] * CUR[i];                         \
        xm_wait<NW>(xm, j & 1, w, lane, (unsigned)j + 1u, f_, E1, E2, a.status, live);              \
        ADJR_PAIRS_NB(CUR, PRV, 0, 2)                                                               \
        if (t + 1 < T) xm_put<NW>(xm, (j + 1) & 1, w, lane, (unsigned)j + 2u, A[0] * PRV[0], A[1] * PRV[1]); \
        __builtin_amdgcn_s_setprio(PT_PRIO_BODY);                                                   \
        ADJR_PAIRS_NB(CUR, PRV, 2, RP)                                                              \
        if (t + 1 < T || last) ADJR_GRAD(CUR, PRV, wv[t], P0, P1, P2)                               \
    }

template <int T, int NW, int RW, bool PROF>
__global__ __launch_bounds__(64 * NW) void k_adj_pr(AdjPtArgs a)
{
    unsigned long long *const prof = PROF ? a.prof : nullptr;   // phase counters: profiled build only
    constexpr bool ADJ_NB = true;                         // barrier-free steps (ADJR_STEP_NB): 1.646 ->
                                                          // 1.577 ms at configs[1] (profiles/r6/adj_nb_ab.txt)
    constexpr bool PT_PRIO = ADJ_NB;                      // wave priorities (PT_PRIO_*)
    constexpr bool PT_MIR = ADJ_NB;                       // mirrored pairs for the exchange's boundary rows
    __shared__ float xch[2][NW][4][64];                   // (the unused exchange is not allocated)
    __shared__ XmBox<NW> xm;                              // the waves' inboxes (xm_*)
    __shared__ double red[64 * NW];
    const TBGeo &g = a.g;
    PT_REGION_INIT(NW, RW)
    const float *AL = a.coeffs + (size_t)b * g.slice;
    f32x2 A[RP], T1v[RP], T2v[RP], L0[RP], L1[RP], GA[RP], GK[RP];   // GA accumulates A x the gradient
    const f32x2 kC2 = {C2, C2}, kC3 = {C3, C3}, kC1X2 = {C1X2, C1X2};
    int srow = -1, rrow = -1;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int gz = wrap_row(uz0 + r, g.Hp);
        const int o = gz * g.ld + gx;
        PT_AT(A, r) = AL[o]; PT_AT(T1v, r) = AL[g.cstride + o]; PT_AT(T2v, r) = AL[2 * g.cstride + o];
        PT_AT(L0, r) = 0.0f; PT_AT(L1, r) = 0.0f;         // L_{nt+1} = L_{nt+2} = 0
        PT_AT(GA, r) = 0.0f; PT_AT(GK, r) = 0.0f;
        if (gz == g.isz && ((rin >> r) & 1u)) srow = r;
        if (gz == g.igz) rrow = r;
    }
    const int isx = g.isx[s];
    const bool scol = xin && gx == isx;
    const float bsrc = srow >= 0 ? AL[4 * g.cstride + (size_t)g.isz * g.ld + isx] : 0.0f;   // beta at the source
    const int rcv0 = rrow >= 0 ? g.rlane[gx] : -1;
    const float *DSb = a.dseis + (size_t)bs * g.nrec * g.dstride;
    const __amdgpu_buffer_rsrc_t DSR = rsrc_of(DSb);
    // source / receiver rows as (row pair, half): a step touches one pair, not all eight rows
    const int spair = __builtin_amdgcn_readfirstlane(srow < 0 ? 0 : PT_MIR ? (srow < RP ? srow : R - 1 - srow) : srow % RP);
    const int rpair = __builtin_amdgcn_readfirstlane(rrow < 0 ? 0 : PT_MIR ? (rrow < RP ? rrow : R - 1 - rrow) : rrow % RP);
    const bool shalf = srow >= RP, rhalf = rrow >= RP;   // the half is r >= RP in both pairings
    // the receiver's row pair among the boundary pairs 0, 1 (rlo) or the interior ones (rhi): wave-uniform
    const int rlo = __builtin_amdgcn_readfirstlane(rrow >= 0 && rpair < 2 ? 1 : 0);
    const int rhi = __builtin_amdgcn_readfirstlane(rrow >= 0 && rpair >= 2 ? 1 : 0);
#define DLOAD(KK)                                                                                   \
    ({                                                                                              \
        const int ri_ = (KK) >= 1 ? rec_index((KK) - 1, g.st) : -1;                                 \
        const bool ok_ = rcv0 >= 0 && ri_ >= 0;                                                     \
        const float v_ = bload(DSR, ok_ ? (ri_ * g.dstride + rcv0) * 4 : OOB, 0);                   \
        ok_ ? v_ : -0.0f;                                                                           \
    })
    const bool grad = rin != 0;                           // uniform: this wave has interior rows
    float gbacc = 0.0f;
    const size_t L = g.level;
    const int L4 = (int)(L * 4);                          // bytes per history slot (< 2 GB: resident surveys)
    f32x2 Q0[RP], Q1[RP], Q2[RP], Q3[RP];
    int pr[R];                                            // history offset of (own row r, lane)
#pragma unroll
    for (int r = 0; r < R; ++r)   // every lane (own cells only, halo lanes at OOB: 1.66 -> 1.73 ms)
        pr[r] = grad ? (PT_ROFS(r) + gx) * 4 : OOB;
#pragma unroll
    for (int i = 0; i < RP; ++i) { Q0[i] = 0.0f; Q1[i] = 0.0f; Q2[i] = 0.0f; Q3[i] = 0.0f; }
    // history descriptor of the epoch whose first step is KN: its prefetches read slots
    // KN - 2 .. KN - T - 1, step t at byte offset (T - 1 - t) * L4
#define HIST_RSRC(KN) rsrc_of(a.hist + (ptrdiff_t)((KN) - T - 1) * (ptrdiff_t)L + (ptrdiff_t)so)
    float wv[T], dv[T];
    if (grad) {   // window of the first step k = nt: slots nt + 1, nt, nt - 1
        const __amdgpu_buffer_rsrc_t H0 = rsrc_of(a.hist + (ptrdiff_t)(a.nt - 1) * (ptrdiff_t)L + (ptrdiff_t)so);
        ADJR_LOAD(Q0, H0, 2 * L4)
        ADJR_LOAD(Q1, H0, L4)
        ADJR_LOAD(Q2, H0, 0)
    }
#pragma unroll
    for (int t = 0; t < T; ++t) {
        wv[t] = a.wav[max(a.nt - t - 1, 0)];
        dv[t] = DLOAD(a.nt - t);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);                   // vmcnt(0)
// the next epoch's wavelet samples and receiver residuals, issued after the sweep as vector loads:
// ahead of it the residual loads make the sweep wait for their round trip (1.65 -> 1.78 ms), and the
// wavelet as scalar loads (wav_s) is slower here too, before the sweep (1.64 -> 1.77 ms: an outstanding
// s_load holds every lgkmcnt wait of the LDS exchange) or after it (1.66 ms; profiles/r6/
// presweep_reorder_ab.txt, wav_scalar_ab.txt)
#define ADJ_ISSUE                                                                                   \
    _Pragma("unroll") for (int t = 0; t < T; ++t) {                                                 \
        wv[t] = a.wav[max(kn - t - 1, 0)];                                                          \
        dv[t] = DLOAD(kn - t);                                                                      \
    }
    const int nep = (a.nt + T - 1) / T;
    bool live = true;
    unsigned long long tsw = 0, tst = 0, tpb = 0, tm = prof ? __builtin_amdgcn_s_memrealtime() : 0;
    unsigned long long tfp = 0, npass = 0;                // profile: first-pass latency, sweep passes
    if constexpr (ADJ_NB) {
        xm_init<NW>(xm, w, lane);                         // no flag matches a tag until written
        __syncthreads();
        xm_put<NW>(xm, 0, w, lane, 1u, f32x2{0.0f, 0.0f}, f32x2{0.0f, 0.0f});   // A L_{nt+1} = 0, step 0's tag
    }
#define ADJR_STEP_SEL(...) { if constexpr (ADJ_NB) ADJR_STEP_NB(__VA_ARGS__) else ADJR_STEP(__VA_ARGS__) }
    for (int e = 0; e < nep; ++e) {
        const int ke = a.nt - e * T;                      // first step k of this epoch
        const bool last = e + 1 == nep;
        const __amdgpu_buffer_rsrc_t HRe = HIST_RSRC(ke);
        // every step of the epoch prefetches a history slot that exists (k >= 2): one scalar test per
        // epoch instead of per step (the barrier-free step, ADJR_STEP_NB)
        int ldall = grad && ke >= T + 1;
        LAUNDER(ldall);
#pragma unroll
        for (int t = 0; t < T; ++t) {
            const int j = e * T + t;
            if (j >= a.nt) break;
            const int k = ke - t;
            if ((t & 3) == 0) ADJR_STEP_SEL(L1, L0, Q0, Q1, Q2, Q3)
            else if ((t & 3) == 1) ADJR_STEP_SEL(L0, L1, Q1, Q2, Q3, Q0)
            else if ((t & 3) == 2) ADJR_STEP_SEL(L1, L0, Q2, Q3, Q0, Q1)
            else ADJR_STEP_SEL(L0, L1, Q3, Q0, Q1, Q2)
        }
        if (T & 1) {   // keep "L1 = newest" at every epoch boundary
#pragma unroll
            for (int i = 0; i < RP; ++i) { const f32x2 tl = L0[i]; L0[i] = L1[i]; L1[i] = tl; }
        }
        // the last step's window (step T - 1: Q[T-1], Q[T], Q[T+1] mod 4), for the deferred gradient
#define QW(o) (((T - 1 + (o)) & 3) == 0 ? Q0 : ((T - 1 + (o)) & 3) == 1 ? Q1 : ((T - 1 + (o)) & 3) == 2 ? Q2 : Q3)
        PT_PROF(tst)
        if (!last) {
            const unsigned tag = (unsigned)(e + 1);
            const __amdgpu_buffer_rsrc_t GR = rsrc_of(a.gran + (size_t)(2 * ((e + 1) & 1)) * L + 2 * so);
            PT_PUBLISH(GR, tag, L0, L1)
            ADJR_GRAD(L0, L1, wv[T - 1], QW(0), QW(1), QW(2))   // the deferred last step (no neighbour data)
            const int kn = ke - T;                        // first step k of the next epoch
            PT_PROF(tpb)
            PT_SWEEP_DELAY()
            PT_SWEEP(GR, tag, L0, L1, PT_ADJ_SG)
            if constexpr (ADJ_NB)   // the next step's boundary rows, with the halo cells the sweep reloaded
                xm_put<NW>(xm, (e + 1) * T & 1, w, lane, (unsigned)((e + 1) * T) + 1u, A[0] * L1[0], A[1] * L1[1]);
            ADJ_ISSUE
            PT_PROF(tsw)
        }
        if constexpr ((T & 3) != 0) {   // restore Q0 = the next epoch's P_k
#pragma unroll
            for (int i = 0; i < RP; ++i) {
                const f32x2 a0 = QW(1)[i], a1 = QW(2)[i], a2 = QW(3)[i], a3 = QW(4)[i];
                Q0[i] = a0; Q1[i] = a1; Q2[i] = a2; Q3[i] = a3;
            }
        }
    }
#undef ADJR_STEP_SEL
#undef QW
#undef DLOAD
#undef ADJ_ISSUE
#undef HIST_RSRC
    if (prof && lane == 0) {
        atomicAdd(prof + 0, tsw); atomicAdd(prof + 1, tst); atomicAdd(prof + 2, tpb); atomicAdd(prof + 3, 1ull);
        atomicAdd(prof + 4, tfp); atomicAdd(prof + 5, npass);
        if (blockIdx.x < PROF_WAVES / 16) {
            unsigned long long *raw = prof + PROF_RAW + ((size_t)blockIdx.x * 16 + w) * 3;   // per wave
            raw[0] = tsw; raw[1] = tst; raw[2] = tpb;
        }
    }
    double ksum = 0.0;                                    // gk = sum K * (sum_k P (L_{k+1} - L_k))
    if (xin) {
#pragma unroll
        for (int r = 0; r < R; ++r)
            if ((rin >> r) & 1u) {
                a.gA[so + (size_t)PT_ROFS(r) + gx] = PT_AT(GA, r) / PT_AT(A, r);
                const float kp = AL[3 * g.cstride + PT_ROFS(r) + gx];
                ksum += (double)kp * (double)PT_AT(GK, r);
            }
    }
    if (srow >= 0 && scol) a.gbeta[bs] = gbacc;
    // deterministic workgroup reduction of the sponge-coefficient partial sum
    const int tid = threadIdx.x;
    red[tid] = ksum;
    __syncthreads();
    for (int w2 = 512; w2 > 0; w2 >>= 1) {
        if (tid < w2 && tid + w2 < 64 * NW) red[tid] += red[tid + w2];
        __syncthreads();
    }
    if (tid == 0) a.gk_part[(size_t)bs * a.nblk + tile] = red[0];
}
#undef ADJR_STEP
#undef FWD_STEP_NB
#undef FWD_PAIRS_NB
#undef MIR_VERT
#undef ADJR_GRAD
#undef ADJR_LOAD
#undef ADJ_STEP
#undef ADJ_GRAD
#undef ADJ_PLOAD
#undef PAIR_VERT
#undef PT_AT
#undef PT_SWEEP
#undef PT_PUBLISH
#undef PT_PROF
#undef PT_SWEEP_DELAY
#undef PT_ROFS
#undef PT_REGION_INIT
#undef PT_REGION_HEAD
#undef PT_REGION_GEOM
#undef LAUNDER
#undef TB_VERT

// Receivers sharing a padded column (ng > nx, or repeated gx): their residuals at one (model, shot,
// record) summed in receiver order into one value per column, the gradient the reference's
// indexing backward builds (index_put with accumulate into zeros, pde.py:82-83), so the time-loop
// kernels inject one value per lane and step with no per-receiver loop.
__global__ __launch_bounds__(256) void k_rcv_fold(const float *__restrict__ ds, float *__restrict__ out,
                                                  const int *__restrict__ colx, const int *__restrict__ rcv_start,
                                                  const int *__restrict__ rcv_list, int ng, int ncolr, size_t rows)
{
    const size_t n = rows * (size_t)ncolr;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const size_t row = i / ncolr;
        const int c = (int)(i - row * ncolr), x = colx[c];
        const float *d = ds + row * ng;
        const int r0 = rcv_start[x], r1 = rcv_start[x + 1];
        float v = d[rcv_list[r0]];
        for (int j = r0 + 1; j < r1; ++j) v = v + d[rcv_list[j]];
        out[i] = v;
    }
}

// --------------------------------------------------------------------------------------- K4
struct FinArgs {
    int B, ns, nz, nx, nbc, Hp, Wp, ld, isz, nblk;
    float dt, dx;
    double scale;     // d(v)/d(input): 1500 for normalised input, 1 for physical velocity
    size_t cstride, slice;
    const float *coeffs, *gA, *gbeta, *vmin;
    const int64_t *amin;
    const double *gk_part;
    const int *isx;
    double *colsum;   // [B][Hp][nx]
    float *out;       // [B][nz][nx]
};

// Stage 1: per padded row z and model column ix, sum g_vpad over the padded columns that
// replicate ix (F.pad replicate backward).  g_vpad is formed per point exactly as autograd
// chains it: alpha = (v*dt/dx)^2 -> ((gA*(2*a1))/dx)*dt; beta = (v*dt)^2 at the sources;
// the sponge term sum(gK*K)/vmin lands on the first argmin of the padded field.
// One workgroup per padded row (z, b): every padded cell's d(loss)/d(v_pad) (fp64) into LDS, all
// cells in parallel; then the replicate-pad fold along x: interior columns take their own cell,
// the two edge columns sum their nbc+1-wide strips (one wave each, fixed-order shuffle tree).
constexpr int FIN_MAXW = 4096;
__global__ __launch_bounds__(256) void k_fin_rows(FinArgs p)
{
    __shared__ double gv_s[FIN_MAXW];
    const int z = blockIdx.x, b = blockIdx.y;
    const size_t ro = (size_t)b * p.slice + (size_t)z * p.ld;
    const float *GA = p.gA + (size_t)b * p.ns * p.slice + (size_t)z * p.ld;   // [B][ns][Hp][ld]
    const float *V = p.coeffs + 5 * p.cstride + ro;
    const int amz = (int)(p.amin[b] / p.nx), amx = (int)(p.amin[b] - (int64_t)amz * p.nx);
    const int apz = amz == 0 ? 0 : amz + p.nbc, apx = amx == 0 ? 0 : amx + p.nbc;
    // sponge term sum(gk_part) of the argmin row: a fixed-order two-level fp64 sum (256 contiguous
    // segments, then the segment sums in order) instead of one thread's serial loop of dependent
    // loads (ns * nblk round trips)
    __shared__ double gk_s[256];
    if (z == apz) {
        const int cnt = p.ns * p.nblk, per = (cnt + 255) / 256;
        const double *GK = p.gk_part + (size_t)b * cnt;
        double acc = 0.0;
        const int j0 = threadIdx.x * per, j1 = min(cnt, j0 + per);
        for (int j = j0; j < j1; j += 4) {
            double v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = GK[min(j + u, cnt - 1)];   // independent loads
#pragma unroll
            for (int u = 0; u < 4; ++u) if (j + u < j1) acc += v[u];
        }
        gk_s[threadIdx.x] = acc;
    }
    __syncthreads();
    for (int x = threadIdx.x; x < p.Wp; x += blockDim.x) {
        float a1 = V[x] * p.dt; a1 = a1 / p.dx;
        float ga = 0.0f;
        {   // shots in order (the oracle's order); the loads are issued 4 at a time
            int s = 0;
            for (; s + 4 <= p.ns; s += 4) {
                float v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) v[u] = GA[(size_t)(s + u) * p.slice + x];
#pragma unroll
                for (int u = 0; u < 4; ++u) ga = ga + v[u];
            }
            for (; s < p.ns; ++s) ga = ga + GA[(size_t)s * p.slice + x];
        }
        float t = ga * (2.0f * a1); t = t / p.dx; t = t * p.dt;
        double gv = (double)t;
        if (z == p.isz) {
            for (int s = 0; s < p.ns; ++s)
                if (p.isx[s] == x) {
                    const float b1 = V[x] * p.dt;
                    float u = p.gbeta[b * p.ns + s] * (2.0f * b1); u = u * p.dt;
                    gv += (double)u;
                }
        }
        if (z == apz && x == apx) {
            double gk = 0.0;
            for (int j = 0; j < 256; ++j) gk += gk_s[j];
            gv += gk / (double)p.vmin[b];
        }
        gv_s[x] = gv;
    }
    __syncthreads();
    double *CS = p.colsum + ((size_t)b * p.Hp + z) * p.nx;
    for (int ix = 1 + threadIdx.x; ix < p.nx - 1; ix += blockDim.x) CS[ix] = gv_s[ix + p.nbc];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (w < 2) {   // wave 0: columns [0, nbc] -> ix 0; wave 1: [nbc+nx-1, Wp) -> ix nx-1
        const int x0 = w == 0 ? 0 : p.nbc + p.nx - 1, x1 = w == 0 ? p.nbc + 1 : p.Wp;
        double acc = 0.0;
        for (int x = x0 + lane; x < x1; x += 64) acc += gv_s[x];
        for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
        if (lane == 0) {
            if (p.nx == 1) { if (w == 0) { double t2 = acc; for (int x = p.nbc + 1; x < p.Wp; ++x) t2 += gv_s[x]; CS[0] = t2; } }
            else CS[w == 0 ? 0 : p.nx - 1] = acc;
        }
    }
}
__global__ __launch_bounds__(256) void k_fin_cols(FinArgs p)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int b = blockIdx.y;
    if (i >= p.nz * p.nx) return;
    const int iz = i / p.nx, ix = i - iz * p.nx;
    const int z0 = iz == 0 ? 0 : iz + p.nbc;
    const int z1 = iz == p.nz - 1 ? p.Hp : iz + p.nbc + 1;
    // the first / last model rows fold nbc + 1 padded rows (121 at OpenFWI): loads issued 16 at a time,
    // then added in row order (the same sum bit for bit; one dependent load per row made this 31 us)
    const double *cs = p.colsum + (size_t)b * p.Hp * p.nx + ix;
    double acc = 0.0;
    int z = z0;
    for (; z + 16 <= z1; z += 16) {
        double v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) v[u] = cs[(size_t)(z + u) * p.nx];
#pragma unroll
        for (int u = 0; u < 16; ++u) acc += v[u];
    }
    for (; z < z1; ++z) acc += cs[(size_t)z * p.nx];
    p.out[(size_t)b * p.nz * p.nx + i] = (float)(acc * p.scale);
}

// --------------------------------------------------------------------------------------- K5
constexpr int L1_BLOCK = 256;
constexpr int L1_ITEMS = 16;   // elements per thread per block tile

__device__ __forceinline__ double block_sum(double v, double *sh)
{
    const int t = threadIdx.x;
    sh[t] = v;
    __syncthreads();
    for (int w = blockDim.x / 2; w > 0; w >>= 1) {
        if (t < w) sh[t] += sh[t + w];
        __syncthreads();
    }
    const double r = sh[0];
    __syncthreads();
    return r;
}

// pass 1: per (model, chunk) partial sums of |y - pred| * mask and of mask (fp64, fixed order)
__global__ __launch_bounds__(L1_BLOCK) void k_l1_partial(int64_t n, const float *__restrict__ pred,
                                                         const float *__restrict__ y,
                                                         const float *__restrict__ mask,
                                                         double *__restrict__ part, int nchunk)
{
    __shared__ double sh[L1_BLOCK];
    const int b = blockIdx.y, c = blockIdx.x;
    const int64_t base = (int64_t)b * n;
    const int64_t c0 = (int64_t)c * L1_BLOCK * L1_ITEMS;
    double se = 0.0, sm = 0.0;
    float dv[L1_ITEMS], mv[L1_ITEMS];
#pragma unroll
    for (int k = 0; k < L1_ITEMS; ++k) {      // all loads first (clamped index, no branch per element)
        const int64_t j = min(c0 + (int64_t)k * L1_BLOCK + threadIdx.x, n - 1);
        mv[k] = mask ? mask[base + j] : 1.0f;
        dv[k] = fabsf(y[base + j] - pred[base + j]);
    }
#pragma unroll
    for (int k = 0; k < L1_ITEMS; ++k) {
        const int64_t j = c0 + (int64_t)k * L1_BLOCK + threadIdx.x;
        if (j < n) {
            se += (double)(dv[k] * mv[k]);
            sm += (double)mv[k];
        }
    }
    se = block_sum(se, sh);
    sm = block_sum(sm, sh);
    if (threadIdx.x == 0) {
        part[((size_t)b * nchunk + c) * 2] = se;
        part[((size_t)b * nchunk + c) * 2 + 1] = sm;
    }
}

// pass 2: one workgroup per model; thread t sums chunks t, t + 256, ... in chunk order, then a fixed
// tree (deterministic).  (One thread per model summed 11.7 k chunks serially at configs[4]: 250 us.)
__global__ __launch_bounds__(L1_BLOCK) void k_l1_final(int B, int nchunk, const double *__restrict__ part,
                                                       float *loss, float *nobs)
{
    __shared__ double sh[L1_BLOCK];
    const int b = blockIdx.x;
    const double *pb = part + (size_t)b * nchunk * 2;
    double se = 0.0, sm = 0.0;
    int c = threadIdx.x;
    for (; c + 7 * L1_BLOCK < nchunk; c += 8 * L1_BLOCK) {   // eight independent loads in flight
        double e[8], m[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) { e[u] = pb[(c + u * L1_BLOCK) * 2]; m[u] = pb[(c + u * L1_BLOCK) * 2 + 1]; }
#pragma unroll
        for (int u = 0; u < 8; ++u) { se += e[u]; sm += m[u]; }
    }
    for (; c < nchunk; c += L1_BLOCK) { se += pb[c * 2]; sm += pb[c * 2 + 1]; }
    se = block_sum(se, sh);
    sm = block_sum(sm, sh);
    if (threadIdx.x == 0) {
        const float no = fmaxf((float)sm, 1.0f);
        nobs[b] = no;
        loss[b] = (float)(se / (double)no);
    }
}

__global__ __launch_bounds__(256) void k_l1_backward(int B, int64_t n, const float *__restrict__ pred,
                                                     const float *__restrict__ y,
                                                     const float *__restrict__ mask,
                                                     const float *__restrict__ nobs,
                                                     const float *__restrict__ gout,
                                                     float *__restrict__ dpred)
{
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int b = blockIdx.y;
    if (j >= n) return;
    const int64_t i = (int64_t)b * n + j;
    const float g = gout[b] / nobs[b];
    const float m = mask ? mask[i] : 1.0f;
    const float d = pred[i] - y[i];
    const float sg = d > 0.0f ? 1.0f : (d < 0.0f ? -1.0f : 0.0f);
    dpred[i] = sg * (m * g);
}

// --------------------------------------------------------------------------------------- K6
__global__ __launch_bounds__(256) void k_smooth_fwd(int kind, int H, int W, const float *__restrict__ mu,
                                                    float *loss)
{
    __shared__ double sh[256];
    const int b = blockIdx.x;
    const float *m = mu + (size_t)b * H * W;
    double sx = 0.0, sy = 0.0;
    const int n = H * W;
    // each thread's elements in its original order, their loads issued 8 at a time (same sums)
    constexpr int CH = 8;
    for (int base = threadIdx.x; base < n; base += CH * blockDim.x) {
        float c[CH], r[CH], d[CH];
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const int i = base + u * blockDim.x;
            const int z = i / W, x = i - z * W;
            c[u] = i < n ? m[i] : 0.0f;
            r[u] = (i < n && x + 1 < W) ? m[i + 1] : 0.0f;
            d[u] = (i < n && z + 1 < H) ? m[i + W] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < CH; ++u) {
            const int i = base + u * blockDim.x;
            if (i >= n) break;
            const int z = i / W, x = i - z * W;
            if (x + 1 < W) { const float e = r[u] - c[u]; sx += kind == 0 ? (double)fabsf(e) : (double)(e * e); }
            if (z + 1 < H) { const float e = d[u] - c[u]; sy += kind == 0 ? (double)fabsf(e) : (double)(e * e); }
        }
    }
    sx = block_sum(sx, sh);
    sy = block_sum(sy, sh);
    if (threadIdx.x == 0) {
        const float tx = (float)(sx / (double)((size_t)H * (W - 1)));
        const float ty = (float)(sy / (double)((size_t)(H - 1) * W));
        loss[b] = tx + ty;
    }
}

__global__ __launch_bounds__(256) void k_smooth_bwd(int kind, int H, int W, const float *__restrict__ mu,
                                                    const float *__restrict__ gout, float *__restrict__ grad)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int b = blockIdx.y;
    if (i >= H * W) return;
    const float *m = mu + (size_t)b * H * W;
    const int z = i / W, x = i - z * W;
    const float gx = gout[b] / (float)((size_t)H * (W - 1));
    const float gy = gout[b] / (float)((size_t)(H - 1) * W);
    auto dterm = [&](float d, float g) {
        if (kind == 0) return d > 0.0f ? g : (d < 0.0f ? -g : 0.0f);
        return 2.0f * d * g;
    };
    float acc = 0.0f;
    if (x + 1 < W) acc -= dterm(m[i + 1] - m[i], gx);
    if (x > 0) acc += dterm(m[i] - m[i - 1], gx);
    if (z + 1 < H) acc -= dterm(m[i + W] - m[i], gy);
    if (z > 0) acc += dterm(m[i] - m[i - W], gy);
    grad[(size_t)b * H * W + i] = acc;
}

}  // namespace

// ======================================================================================= plan
struct GraphEntry {
    int kind;                 // 0 fwd-history, 1 fwd-ring, 2 adjoint
    int B;
    const void *ptrs[8];
    hipGraphExec_t exec;
    uint64_t last_use;
};

// default pre-sweep delays of the persistent forward / adjoint, 10 ns ticks (PT_SWEEP_DELAY)
constexpr int RDQ_SWEEP_DELAY_FWD = 15, RDQ_SWEEP_DELAY_ADJ = 0;

struct rdq_fwi_plan {
    rdq_fwi_geom g;
    std::vector<int32_t> isx, igx;
    std::vector<double> wav;
    std::vector<float> wavf;
    int Hp, Wp, ld, nrec;
    int *d_isx = nullptr, *d_rcv_start = nullptr, *d_rcv_list = nullptr;
    int *d_rlane = nullptr;     // [Wp] adjoint residual index per column (receiver id, or folded column)
    int *d_colx = nullptr;      // [ncolr] padded column of each receiver column (fold)
    int ncolr = 0;              // columns holding a receiver
    bool rmulti = false;        // some column holds several receivers: residuals folded per column
    float *d_wav = nullptr;     // fp32 wavelet [nt] (persistent kernels)
    unsigned *d_status = nullptr;   // status words in use: d_status_own or a caller buffer (rdq_fwi_set_status_buffer)
    unsigned *d_status_own = nullptr;
    unsigned long long *d_prof = nullptr;   // phase counters (rdq_fwi_set_profile): fwd, then adj
    std::vector<unsigned long long> prof_host;
    bool graphs = true;
    int persist = 1;            // 0 off, 1 auto, 8 / 12: persistent kernels with that region height (waves),
                                // -1: persistent launches oversubscribed 2x past residency (fault-path test)
    int xcd_mode = 1;           // persistent kernels: XCD-local slices with L2 hand-offs (pt_assign)
    // resident workgroups (0 = unknown) per kernel variant [variant][T]: 0 fwd 64-row, 1..3 fwd 96-row
    // with 8 / 12 / 24 rows per wave, 4 exact adjoint 64-row, 5 exact 96-row, 6 FMA adjoint 64-row,
    // 7..8 FMA adjoint 96-row with 8 / 12 rows per wave
    int capw[13][TB_MAXT + 1] = {};   // [9] fwd 96-row x 6 rows per wave, [10] FMA adjoint 96-row x 6,
                                      // [11] / [12] fwd / FMA adjoint 64-row x 4 rows per wave (class 16)
    int fwd_rw = 6, adj_rw = 6;   // rows per wave of the 96-row persistent kernels (rdq_fwi_set_rows_per_wave;
                                  // adjoint 6: 1.649 vs 1.672 ms for 8, profiles/r3/adj_rows_nb_ab.txt)
    int fwd_T = 4, adj_T = 4;   // time steps per launch (temporal blocking depth), <= TB_MAXT
    int fwd_delay = RDQ_SWEEP_DELAY_FWD, adj_delay = RDQ_SWEEP_DELAY_ADJ;   // persistent kernels' pre-sweep delay (ticks)
    int adj_Tw = 0;             // the wide chunked adjoint's depth (<= TW_ADJ_MAXT); 0 = auto, see wide_adj_depth
    int fwd_Tw = 0;             // the wide chunked forward's depth (<= TW_FWD_MAXT); 0 = auto, see wide_fwd_depth
    int adj_spw = 0;            // the wide chunked adjoint's shots per workgroup, 0 = auto (wide_spw)
    int fwd_spw = 0;            // the wide chunked forward's, 0 = auto
    int chains = 0;             // independent shot groups launched as concurrent chains; 0 = auto (chain_count)
    bool fwd_gen = true;        // chunked forward regenerates coefficients from the model (vs loading K3)
    bool adj_fma = true;        // persistent adjoint with FMA contraction (vs the oracle's exact op order)
    bool adj_tw_fma = false;    // wide chunked adjoint with FMA contraction (RDQ_VARIANT_CHUNKED_ADJ_FMA; default:
                                // the oracle's exact order, bitwise gA / gbeta / gk terms)
    bool wide = true;           // chunked kernels on 128-column regions (k_fwd_tw / k_adj_tw) vs 64-column
    hipStream_t cap = nullptr;
    std::vector<hipStream_t> aux;
    std::vector<hipEvent_t> evs;   // [0] fork, [1..] joins (inside graph capture: graph edges)
    std::vector<GraphEntry> cache;
    uint64_t tick = 0;
    // One call in flight per plan: the host state above (graph cache, chain streams and events) is
    // guarded by `mu`, and a time-loop call on another stream than the previous one first waits on an
    // event recorded on that stream at this point (`handover`), so calls on one plan from several
    // streams run one after the other on the device (the persistent launches share the plan's arrival
    // counters and each needs the whole chip; the chunked launches share the chain streams).
    std::mutex mu;
    hipStream_t last = nullptr;
    bool have_last = false;
    hipEvent_t handover = nullptr;
};

namespace {

int tiles_x(int Wp, int T) { return (Wp + (64 - 4 * T) - 1) / (64 - 4 * T); }
int tiles_y(int Hp, int T) { return (Hp + (TB_RH - 4 * T) - 1) / (TB_RH - 4 * T); }


TBGeo tb_geo(const rdq_fwi_plan *p, int B)
{
    TBGeo g;
    g.B = B; g.ns = p->g.ns; g.Hp = p->Hp; g.Wp = p->Wp; g.ld = p->ld;
    g.isz = p->g.isz; g.igz = p->g.igz; g.ng = p->g.ng; g.nrec = p->nrec; g.st = p->g.sample_temporal;
    g.slice = (size_t)p->Hp * p->ld;
    g.cstride = (size_t)B * g.slice;
    g.level = (size_t)B * g.ns * g.slice;
    g.isx = p->d_isx; g.rcv_start = p->d_rcv_start; g.rcv_list = p->d_rcv_list;
    g.rlane = p->d_rlane; g.dstride = p->rmulti ? p->ncolr : p->g.ng;
    g.s_off = 0; g.ns_grp = p->g.ns;
    g.sl_off = 0; g.nsl = B * p->g.ns;
    return g;
}

// Shots split into `chains` groups, each a dependent chain of launches on its own stream, forked
// from and joined back into `st` with events (inside graph capture this records parallel graph
// branches).  Concurrent chains overlap each launch's fixed latency (prologue loads, store
// drain, dispatch) with the other chains' compute.
// Concurrent launch chains of a chunked time loop.  Auto: two for the wide kernels (each chain's
// launches fill the other's tail rounds: configs[4] forward 54.7 -> 49.0-50.0 ms, adjoint 93.8 ->
// 91.0-91.6; 3 / 4 / 8 chains 51.7 / 53.9 / 58.0 and 93.1 / 95.1 / 101.2; profiles/r5/configs4_chains.jsonl),
// one for the 64-column kernels.
int chain_count(const rdq_fwi_plan *p)
{
    const int c = p->chains > 0 ? p->chains : (p->wide ? 2 : 1);
    return std::max(1, std::min(c, p->g.ns));
}

// Default depth of the wide chunked adjoint, measured at configs[4] (profiles/r5/configs4_wide_adj_depth.jsonl):
// 5 steps per launch is the fastest for both forms (exact order 116.1-116.3 ms vs 120.4 at 4 and 120.6
// at 6; contracted 111.2 ms vs 115.1-115.7 at 6).
constexpr int TW_ADJ_DEFAULT = 5;
int wide_adj_depth(const rdq_fwi_plan *p) { return p->adj_Tw > 0 ? p->adj_Tw : TW_ADJ_DEFAULT; }
// Default depth of the wide chunked forward: rdq_fwi_set_tuning's fwd_steps (the persistent kernels'
// depth, <= 4) unless rdq_fwi_set_wide_fwd_steps chose one (<= TW_FWD_MAXT)
int wide_fwd_depth(const rdq_fwi_plan *p) { return p->fwd_Tw > 0 ? p->fwd_Tw : p->fwd_T; }

// Compute units of the device the plan's launches run on, cached per device (a process may drive
// several GPUs; the count is queried once per device id).
int device_cus()
{
    constexpr int MAXDEV = 64;
    static std::atomic<int> cache[MAXDEV];               // 0 = not queried yet
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (dev >= 0 && dev < MAXDEV && (n = cache[dev].load(std::memory_order_relaxed)) > 0) return n;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1) n = 256;
    if (dev >= 0 && dev < MAXDEV) cache[dev].store(n, std::memory_order_relaxed);
    return n;
}

// Shots per workgroup of a wide forward / adjoint launch over `regions` (models x tiles) of `ns` shots.  A
// workgroup generates its region's coefficients once for all its shots and pays its fixed start-up
// once, so more is cheaper per shot, but a workgroup of many shots is a long indivisible unit.  Cost
// model: rounds of one workgroup per CU x (shots per workgroup + kappa), kappa = a workgroup's fixed
// cost in shots, fitted at configs[4] (profiles/r5/configs4_adj_spw.jsonl, configs4_fwd_spw.jsonl):
// forward 0.6, adjoint 0.25; the cheapest of 16 / 8 / 4 / 2 / 1 (ties: more shots).  `chains` launch
// chains run concurrently and share the CUs, so one chain's launch gets cus / chains of them.
// configs[4] (16 shots in two chains of 8, 203 forward / 510 adjoint regions): 8 for both; with one
// chain, 16 for both (forward 57.5 -> 54.9 ms, adjoint 94.9 -> 94.1 against 8: configs4_spw16.jsonl); a
// small grid (20 regions) keeps 1 for parallelism.
int wide_spw(int setting, int regions, int ns, bool adj, int chains)
{
    if (setting > 0) return std::max(1, std::min(setting, ns));
    const int cus = std::max(1, device_cus() / std::max(1, chains));
    const double kappa = adj ? 0.25 : 0.6;
    int pick = 1;
    double best = 1e300;
    for (const int c : {16, 8, 4, 2, 1}) {
        const int spw = std::min(c, ns), groups = (ns + spw - 1) / spw;
        const long long wgs = (long long)regions * groups, rounds = (wgs + cus - 1) / cus;
        const double cost = (double)rounds * (spw + kappa);
        if (cost < best - 1e-9) { best = cost; pick = spw; }
    }
    return pick;
}

// A time-loop call on `st` (caller holds p->mu): when the plan's previous call went to another
// stream, `st` first waits for everything that stream had queued by now (which includes that call),
// so calls on one plan never overlap on the device whatever streams they come on.  A steady caller
// (one stream) pays nothing.  Skipped while either stream is being captured into a graph: a captured
// stream cannot wait on an event recorded outside the capture (the caller orders captured work).
int plan_enter(rdq_fwi_plan *p, hipStream_t st)
{
    if (p->have_last && p->last != st) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone, cl = hipStreamCaptureStatusNone;
        RDQ_CHECK(hipStreamIsCapturing(st, &cs));
        RDQ_CHECK(hipStreamIsCapturing(p->last, &cl));
        if (cs == hipStreamCaptureStatusNone && cl == hipStreamCaptureStatusNone) {
            if (!p->handover) RDQ_CHECK(hipEventCreateWithFlags(&p->handover, hipEventDisableTiming));
            RDQ_CHECK(hipEventRecord(p->handover, p->last));
            RDQ_CHECK(hipStreamWaitEvent(st, p->handover, 0));
        }
    }
    p->last = st;
    p->have_last = true;
    return 0;
}

// The chunked adjoints accumulate each workgroup's sponge partial into gk_part[(b * ns + shot) * nblk
// + tile]: the narrow kernel with a load-add-store, the wide one with a no-return fp64 atomic add.  Both
// are deterministic (and the load-add-store race-free) only if every slot has ONE writer per launch
// (the adds of a slot then arrive launch after launch, in stream order) and no slot is written by two
// concurrent launch chains.  GkWriters replays the kernels' own block decode (decode_tile, the
// shot-group split of k_adj_tw / k_adj_tb) for every launch of a time loop on the host, when the loop
// is enqueued (once per captured graph), and refuses the call (RDQ_E_INVALID) on a violation or on a
// slot outside the caller's gk_part buffer.
struct GkWriters {
    std::vector<int> chain;          // chain that owns the slot (-1: none yet)
    std::vector<unsigned> stamp;     // last launch that wrote it
    unsigned launch = 0;
    int nblk;
    GkWriters(size_t slices, int nblk_) : chain(slices * nblk_, -1), stamp(slices * nblk_, 0u), nblk(nblk_) {}
    // one launch of chain c: grid blocks, tile grid, B models x ns shots, shot group [s_off, s_off + ns_sh)
    // split in groups of spw shots (ns_grp groups)
    bool add(int c, unsigned grid, int tiles_x, int ntiles, int B, int ns, int ns_grp, int s_off, int spw, int ns_sh)
    {
        ++launch;
        const int nsg = B * ns_grp;
        for (unsigned L = 0; L < grid; ++L) {
            const TileId ti = decode_tile((int)L, tiles_x, ntiles, nsg);
            if (!ti.valid) continue;
            if (ti.tile >= nblk) return false;
            const int b = ti.sl / ns_grp, jg = ti.sl - b * ns_grp;
            const int s_first = s_off + jg * spw, nsh = std::min(spw, ns_sh - jg * spw);
            for (int sh = 0; sh < nsh; ++sh) {
                const size_t slot = (size_t)(b * ns + s_first + sh) * nblk + ti.tile;
                if (s_first + sh >= ns || slot >= chain.size()) return false;
                if (stamp[slot] == launch || (chain[slot] >= 0 && chain[slot] != c)) return false;
                stamp[slot] = launch;
                chain[slot] = c;
            }
        }
        return true;
    }
};

int ensure_aux(rdq_fwi_plan *p, int S)
{
    while ((int)p->aux.size() < S - 1) {
        hipStream_t s;
        RDQ_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        p->aux.push_back(s);
    }
    while ((int)p->evs.size() < S) {
        hipEvent_t e;
        RDQ_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        p->evs.push_back(e);
    }
    return 0;
}

int fork_chains(rdq_fwi_plan *p, hipStream_t st, int S)
{
    if (S == 1) return 0;
    RDQ_TRY(ensure_aux(p, S));
    RDQ_CHECK(hipEventRecord(p->evs[0], st));
    for (int c = 1; c < S; ++c) RDQ_CHECK(hipStreamWaitEvent(p->aux[c - 1], p->evs[0], 0));
    return 0;
}

int join_chains(rdq_fwi_plan *p, hipStream_t st, int S)
{
    for (int c = 1; c < S; ++c) {
        RDQ_CHECK(hipEventRecord(p->evs[c], p->aux[c - 1]));
        RDQ_CHECK(hipStreamWaitEvent(st, p->evs[c], 0));
    }
    return 0;
}

// coeffs buffer: [6][B][Hp][ld] fields, then v_model [B][nz][nx], then ks [B]
CoefGen coef_gen(const rdq_fwi_plan *p, int B, const float *coeffs)
{
    CoefGen c;
    const size_t cstride = (size_t)B * p->Hp * p->ld;
    c.vmod = coeffs + 6 * cstride;
    c.ks = c.vmod + (size_t)B * p->g.nz * p->g.nx;
    c.nz = p->g.nz; c.nx = p->g.nx; c.nbc = p->g.nbc; c.Hp = p->Hp; c.Wp = p->Wp;
    c.dt = p->g.dt; c.dx = p->g.dx;
    c.a = (float)((double)(p->g.nbc - 1) * (double)p->g.dx);
    return c;
}

template <int TT, bool G>
void launch_fwd1(dim3 grid, hipStream_t st, const FwdTBArgs &a)
{
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_fwd_tb<TT, G>), grid, dim3(64 * TB_NW), 0, st, a);
}

void launch_fwd(int T, bool gen, dim3 grid, hipStream_t st, const FwdTBArgs &a)
{
    switch (T * 2 + (gen ? 1 : 0)) {
    case 2: launch_fwd1<1, false>(grid, st, a); break;
    case 3: launch_fwd1<1, true>(grid, st, a); break;
    case 4: launch_fwd1<2, false>(grid, st, a); break;
    case 5: launch_fwd1<2, true>(grid, st, a); break;
    case 6: launch_fwd1<3, false>(grid, st, a); break;
    case 7: launch_fwd1<3, true>(grid, st, a); break;
    case 8: launch_fwd1<4, false>(grid, st, a); break;
    default: launch_fwd1<4, true>(grid, st, a); break;
    }
}

template <class Args>
void launch_adj(int T, dim3 grid, hipStream_t st, const Args &a)
{
    const dim3 blk(64 * TB_NW);
    switch (T) {
    case 1: hipLaunchKernelGGL(k_adj_tb<1>, grid, blk, 0, st, a); break;
    case 2: hipLaunchKernelGGL(k_adj_tb<2>, grid, blk, 0, st, a); break;
    case 3: hipLaunchKernelGGL(k_adj_tb<3>, grid, blk, 0, st, a); break;
    default: hipLaunchKernelGGL(k_adj_tb<4>, grid, blk, 0, st, a); break;
    }
}

// wide chunked regions: forward 16 waves x 8 rows (128 x 128), adjoint 16 waves x 4 rows (128 x 64:
// its seven two-column fields per row fill the 128 VGPRs of a 1024-thread workgroup)
constexpr int TW_FWD_NW = 16, TW_FWD_R = 8, TW_ADJ_NW = 16, TW_ADJ_R = 4;
static_assert(ADJ_W_MAX >= TW_ADJ_MAXT && ADJ_W_MAX >= TB_MAXT, "AdjTBArgs::w holds one sample per step of a launch");
int tw_tiles_x(int Wp, int T) { return (Wp + (TW_W - 4 * T) - 1) / (TW_W - 4 * T); }
int tw_tiles_y(int Hp, int T, bool adj)
{
    const int ih = (adj ? TW_ADJ_NW * TW_ADJ_R : TW_FWD_NW * TW_FWD_R) - 4 * T;
    return (Hp + ih - 1) / ih;
}

template <int TT>
void launch_fwd_w_T(bool gen, bool pair, dim3 grid, hipStream_t st, const FwdTBArgs &a)
{
    const dim3 blk(64 * TW_FWD_NW);
    if (gen) {
        if (pair) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_fwd_tw<TT, TW_FWD_NW, TW_FWD_R, true, true>), grid, blk, 0, st, a);
        else hipLaunchKernelGGL(HIP_KERNEL_NAME(k_fwd_tw<TT, TW_FWD_NW, TW_FWD_R, true, false>), grid, blk, 0, st, a);
    } else {
        if (pair) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_fwd_tw<TT, TW_FWD_NW, TW_FWD_R, false, true>), grid, blk, 0, st, a);
        else hipLaunchKernelGGL(HIP_KERNEL_NAME(k_fwd_tw<TT, TW_FWD_NW, TW_FWD_R, false, false>), grid, blk, 0, st, a);
    }
}
void launch_fwd_w(int T, bool gen, bool pair, dim3 grid, hipStream_t st, const FwdTBArgs &a)
{
    switch (T) {
    case 1: launch_fwd_w_T<1>(gen, pair, grid, st, a); break;
    case 2: launch_fwd_w_T<2>(gen, pair, grid, st, a); break;
    case 3: launch_fwd_w_T<3>(gen, pair, grid, st, a); break;
    case 4: launch_fwd_w_T<4>(gen, pair, grid, st, a); break;
    case 5: launch_fwd_w_T<5>(gen, pair, grid, st, a); break;
    default: launch_fwd_w_T<6>(gen, pair, grid, st, a); break;
    }
}
static_assert(FWD_W_MAX >= TW_FWD_MAXT && FWD_W_MAX >= TB_MAXT, "FwdTBArgs::w holds one sample per step of a launch");
template <int TT, bool EX>
void launch_adj_w_T(bool pair, dim3 grid, hipStream_t st, const AdjTBArgs &a)
{
    const dim3 blk(64 * TW_ADJ_NW);
    if (pair) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_adj_tw<TT, TW_ADJ_NW, TW_ADJ_R, true, EX>), grid, blk, 0, st, a);
    else hipLaunchKernelGGL(HIP_KERNEL_NAME(k_adj_tw<TT, TW_ADJ_NW, TW_ADJ_R, false, EX>), grid, blk, 0, st, a);
}
void launch_adj_w(int T, bool pair, bool exact, dim3 grid, hipStream_t st, const AdjTBArgs &a)
{
    switch (T * 2 + (exact ? 1 : 0)) {
    case 2: launch_adj_w_T<1, false>(pair, grid, st, a); break;
    case 3: launch_adj_w_T<1, true>(pair, grid, st, a); break;
    case 4: launch_adj_w_T<2, false>(pair, grid, st, a); break;
    case 5: launch_adj_w_T<2, true>(pair, grid, st, a); break;
    case 6: launch_adj_w_T<3, false>(pair, grid, st, a); break;
    case 7: launch_adj_w_T<3, true>(pair, grid, st, a); break;
    case 8: launch_adj_w_T<4, false>(pair, grid, st, a); break;
    case 9: launch_adj_w_T<4, true>(pair, grid, st, a); break;
    case 10: launch_adj_w_T<5, false>(pair, grid, st, a); break;
    case 11: launch_adj_w_T<5, true>(pair, grid, st, a); break;
    case 12: launch_adj_w_T<6, false>(pair, grid, st, a); break;
    default: launch_adj_w_T<6, true>(pair, grid, st, a); break;
    }
}

// Workgroups of a persistent kernel the device holds at once (occupancy query x CUs).
template <class K>
int resident_capacity(K kernel, int nthreads, int &cache)
{
    if (cache) return cache;
    int dev = 0, cus = 0, nb = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -1;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, nthreads, 0) != hipSuccess) return -1;
    cache = cus * nb;
    return cache;
}

// Resident capacity of the persistent kernel a call would launch (occupancy query x CUs).  `NW` is
// the region-height class (region rows = NW x 8: 64 or 96); the 96-row kernels run 8, 12 or 24 rows
// per wave (12, 8 or 4 waves per workgroup).  The adjoint's launch must fit both adjoint variants.
template <int T>
int capacity_T(rdq_fwi_plan *p, int NW, bool adj)
{
    auto *c = p->capw;
    if (!adj) {
        if (NW == 16) return resident_capacity(k_fwd_pt<T, 16, 4, false>, 1024, c[11][T]);
        if (NW != 12) return resident_capacity(k_fwd_pt<T, 8, 8, false>, 512, c[0][T]);
        if (p->fwd_rw == 24) return resident_capacity(k_fwd_pt<T, 4, 24, false>, 256, c[3][T]);
        if (p->fwd_rw == 6) return resident_capacity(k_fwd_pt<T, 16, 6, false>, 1024, c[9][T]);
        if (p->fwd_rw == 12) return resident_capacity(k_fwd_pt<T, 8, 12, false>, 512, c[2][T]);
        return resident_capacity(k_fwd_pt<T, 12, 8, false>, 768, c[1][T]);
    }
    if (NW != 12)
        return std::min(resident_capacity(k_adj_pt<T, 8, false>, 512, c[4][T]),
                        NW == 16 ? resident_capacity(k_adj_pr<T, 16, 4, false>, 1024, c[12][T])
                                 : resident_capacity(k_adj_pr<T, 8, 8, false>, 512, c[6][T]));
    const int ex = resident_capacity(k_adj_pt<T, 12, false>, 768, c[5][T]);
    if (p->adj_rw == 12) return std::min(ex, resident_capacity(k_adj_pr<T, 8, 12, false>, 512, c[8][T]));
    if (p->adj_rw == 6) return std::min(ex, resident_capacity(k_adj_pr<T, 16, 6, false>, 1024, c[10][T]));
    return std::min(ex, resident_capacity(k_adj_pr<T, 12, 8, false>, 768, c[7][T]));
}
int capacity_nw(rdq_fwi_plan *p, int NW, bool adj, int T)
{
    switch (T) {
    case 1: return capacity_T<1>(p, NW, adj);
    case 2: return capacity_T<2>(p, NW, adj);
    case 3: return capacity_T<3>(p, NW, adj);
    default: return capacity_T<4>(p, NW, adj);
    }
}

// Region classes of the persistent kernels: 12 = 64 x 96 regions (the plan's rows per wave),
// 8 = 64 x 64 regions of 8 waves x 8 rows, 16 = 64 x 64 regions of 16 waves x 4 rows.
static int region_rows(int NW) { return NW == 12 ? 96 : 64; }

// tiles (padded to the 8-XCD deal) of one (model, shot) slice at depth T with NW-wave regions
unsigned pt_tiles_padded(const rdq_fwi_plan *p, int T, int NW)
{
    const int ih = region_rows(NW) - 4 * T;
    const int nt_ = tiles_x(p->Wp, T) * ((p->Hp + ih - 1) / ih);
    return (unsigned)((nt_ + 7) / 8 * 8);
}

// Per-(model, shot) slots of the sponge-term partials gk_part: one per tile of whichever kernel runs
// the adjoint (persistent classes, narrow or wide chunked, every depth T), sized to the largest tile
// count over all of them, so no region shape can outgrow the buffer the caller allocated
// (rdq_fwi_sizes) and the finalize sums (k_fin_rows: unused slots stay zero).
int gk_blocks(const rdq_fwi_plan *p)
{
    int n = 0;
    for (int T = 1; T <= TW_ADJ_MAXT; ++T)                                       // wide chunked (128 x 64)
        n = std::max(n, tw_tiles_x(p->Wp, T) * tw_tiles_y(p->Hp, T, true));
    for (int T = 1; T <= TB_MAXT; ++T) {
        n = std::max(n, tiles_x(p->Wp, T) * tiles_y(p->Hp, T));                  // narrow chunked (64 x 64)
        n = std::max(n, tw_tiles_x(p->Wp, T) * tw_tiles_y(p->Hp, T, true));      // wide chunked (128 x 64)
        for (int NW : {8, 12, 16}) {                                             // persistent region classes
            const int ih = region_rows(NW) - 4 * T;
            n = std::max(n, tiles_x(p->Wp, T) * ((p->Hp + ih - 1) / ih));
        }
    }
    return n;
}

// Slices (model x shot) per persistent launch: every slice of one launch must be resident at once,
// so a batch larger than the chip (e.g. 32 OpenFWI shots = 4 x 224 workgroups, or the reference's
// OpenFWI config of 25 models x 5 shots = 125 slices) runs as ceil(B ns / per) launches over
// consecutive runs of the flat slice index b * ns + s, of near-equal size; 0 = not even one slice fits.
int pt_slices_per_launch(const rdq_fwi_plan *p, int B, int T, int NW, int cap)
{
    if (cap <= 0) return 0;
    const unsigned per = (unsigned)cap / pt_tiles_padded(p, T, NW);
    if (per < 1) return 0;
    const int total = B * p->g.ns, groups = (total + (int)per - 1) / (int)per;
    return (total + groups - 1) / groups;
}

// grid of a persistent launch covering S slices.  A slice is XCD-local (L2 hand-offs,
// pt_assign) only if one XCD received all its Tt workgroups; blocks are dealt round-robin over the
// 8 XCDs, so a launch of S slices gets that for every slice only with >= 8 Tt ceil(S / 8) blocks.
// Launches of fewer than 8 slices (e.g. the reference's 5-shot survey: 5 x 32 = 160 blocks, 20 per
// XCD) are padded up to it when the chip holds that many; the surplus blocks find no slice and exit.
unsigned pt_grid(const rdq_fwi_plan *p, int T, int NW, int nsl, bool adj)
{
    const unsigned S = (unsigned)nsl;
    unsigned grid = pt_tiles_padded(p, T, NW) * S;
    if (p->xcd_mode) {
        const int ih = region_rows(NW) - 4 * T;
        const unsigned Tt = (unsigned)(tiles_x(p->Wp, T) * ((p->Hp + ih - 1) / ih));
        const unsigned want = 8u * Tt * ((S + 7u) / 8u);
        const int cap = capacity_nw(const_cast<rdq_fwi_plan *>(p), NW, adj, T);
        if (want > grid && (int)want <= cap) grid = want;
    }
    if (p->persist == -1) {   // fault-path test: a grid the device cannot hold resident at once
        const int cap = capacity_nw(const_cast<rdq_fwi_plan *>(p), NW, adj, T);
        grid = std::max(grid, 2u * (unsigned)std::max(cap, 1));
    }
    return grid;
}

// region height (waves) of the persistent kernel for this call, 0 = not resident -> chunked.
// Taller regions first: one workgroup per CU and less halo (64 x 96 vs 64 x 64).  `per` = slices
// per launch (the batch runs as ceil(B ns / per) launches).
// Small surveys first: a launch of at most PT_SMALL_WG workgroups in 64 x 64 regions of 16 waves x
// 4 rows runs each step with 2/3 of the 96-row kernels' per-wave work on CUs the 96-row launch leaves
// idle (profiles/r3/pt64_ab.txt, configs[1] geometry: 3 shots = 168 workgroups, forward 1.30 -> 1.14
// ms, adjoint 1.65 -> 1.44; at 5 shots, 280, no slice fits one XCD and it is slower).
constexpr unsigned PT_SMALL_WG = 200;
int persistent_nw(rdq_fwi_plan *p, int B, bool adj, int *per = nullptr)
{
    if (!p->persist) return 0;
    const int T = adj ? p->adj_T : p->fwd_T;
    const int want = p->persist == -1 ? 1 : p->persist;   // 1 = auto, 8 / 12 / 16 = forced
    if (want == 1 || want == 16) {
        const int k = pt_slices_per_launch(p, B, T, 16, capacity_nw(p, 16, adj, T));
        const bool small = k >= B * p->g.ns && pt_tiles_padded(p, T, 16) * (unsigned)(B * p->g.ns) <= PT_SMALL_WG;
        if (k > 0 && (want == 16 || small)) { if (per) *per = k; return 16; }
    }
    if (want == 1 || want == 12) {
        const int k = pt_slices_per_launch(p, B, T, 12, capacity_nw(p, 12, adj, T));
        if (k > 0) { if (per) *per = k; return 12; }
    }
    if (want == 1 || want == 8) {
        const int k = pt_slices_per_launch(p, B, T, 8, capacity_nw(p, 8, adj, T));
        if (k > 0) { if (per) *per = k; return 8; }
    }
    return 0;
}

// the persistent forward of region class NW (64 / 96 rows) with the plan's rows per wave
template <int T, bool PROF>
void launch_fwd_pt_T(const rdq_fwi_plan *p, int NW, dim3 grid, hipStream_t st, const FwdPtArgs &a)
{
    if (NW == 16) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_fwd_pt<T, 16, 4, PROF>), grid, dim3(1024), 0, st, a);
    else if (NW != 12) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_fwd_pt<T, 8, 8, PROF>), grid, dim3(512), 0, st, a);
    else if (p->fwd_rw == 24) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_fwd_pt<T, 4, 24, PROF>), grid, dim3(256), 0, st, a);
    else if (p->fwd_rw == 12) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_fwd_pt<T, 8, 12, PROF>), grid, dim3(512), 0, st, a);
    else if (p->fwd_rw == 6) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_fwd_pt<T, 16, 6, PROF>), grid, dim3(1024), 0, st, a);
    else hipLaunchKernelGGL(HIP_KERNEL_NAME(k_fwd_pt<T, 12, 8, PROF>), grid, dim3(768), 0, st, a);
}
void launch_fwd_pt(const rdq_fwi_plan *p, int NW, int T, dim3 grid, hipStream_t st, const FwdPtArgs &a)
{
    if (a.prof && T == 4) { launch_fwd_pt_T<4, true>(p, NW, grid, st, a); return; }   // phase-profiled build
    switch (T) {
    case 1: launch_fwd_pt_T<1, false>(p, NW, grid, st, a); break;
    case 2: launch_fwd_pt_T<2, false>(p, NW, grid, st, a); break;
    case 3: launch_fwd_pt_T<3, false>(p, NW, grid, st, a); break;
    default: launch_fwd_pt_T<4, false>(p, NW, grid, st, a); break;
    }
}

// the persistent adjoint: FMA / recurrence build (k_adj_pr, the plan's rows per wave for 96-row
// regions) or the oracle's exact operation order (k_adj_pt, 8 rows per wave)
template <int T, bool PROF>
void launch_adj_pt_T(const rdq_fwi_plan *p, int NW, dim3 grid, hipStream_t st, const AdjPtArgs &a)
{
    if (!p->adj_fma) {
        if (NW != 12) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_adj_pt<T, 8, PROF>), grid, dim3(512), 0, st, a);
        else hipLaunchKernelGGL(HIP_KERNEL_NAME(k_adj_pt<T, 12, PROF>), grid, dim3(768), 0, st, a);
    } else if (NW == 16) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_adj_pr<T, 16, 4, PROF>), grid, dim3(1024), 0, st, a);
    else if (NW != 12) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_adj_pr<T, 8, 8, PROF>), grid, dim3(512), 0, st, a);
    else if (p->adj_rw == 12) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_adj_pr<T, 8, 12, PROF>), grid, dim3(512), 0, st, a);
    else if (p->adj_rw == 6) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_adj_pr<T, 16, 6, PROF>), grid, dim3(1024), 0, st, a);
    else hipLaunchKernelGGL(HIP_KERNEL_NAME(k_adj_pr<T, 12, 8, PROF>), grid, dim3(768), 0, st, a);
}
void launch_adj_pt(const rdq_fwi_plan *p, int NW, int T, dim3 grid, hipStream_t st, const AdjPtArgs &a)
{
    if (a.prof && T == 4) { launch_adj_pt_T<4, true>(p, NW, grid, st, a); return; }   // phase-profiled build
    switch (T) {
    case 1: launch_adj_pt_T<1, false>(p, NW, grid, st, a); break;
    case 2: launch_adj_pt_T<2, false>(p, NW, grid, st, a); break;
    case 3: launch_adj_pt_T<3, false>(p, NW, grid, st, a); break;
    default: launch_adj_pt_T<4, false>(p, NW, grid, st, a); break;
    }
}

// The buffers a launch needs zeroed (granules, accumulators, history slots, adjoint levels, pt_assign's
// arrival counters) in ONE stream-ordered kernel instead of a memset each (each memset is a separate
// ~5 us dispatch on the step's critical path).  Sizes are multiples of 4 B; 16-byte-aligned regions are
// cleared with 16-byte stores, others with 4-byte ones.
// The chunked launchers run inside hipGraph capture (run_cached), and they must not use
// hipMemsetAsync there: on this ROCm (7.2) the captured memset node (present and first in the chain:
// profiles/r5/graph_replay/captured_memset_node.dot.txt) takes effect on the graph exec's first launch
// but not on its replays, which then read whatever the buffer held (tools/diag_graph_rawmem.py on
// hipMalloc'd buffers; the minimal memset + kernel-chain graphs of tools/repro/graph_kernarg.hip
// replay correctly, so the trigger is not isolated).  The zeroing kernel replays correctly.
constexpr int ZERO_MAXR = 6;
struct ZeroArgs {
    void *p[ZERO_MAXR];
    size_t n[ZERO_MAXR];      // bytes
    int nr;
};
__global__ __launch_bounds__(256) void k_zero_regions(ZeroArgs z)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x, t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (int r = 0; r < z.nr; ++r) {
        if ((reinterpret_cast<uintptr_t>(z.p[r]) & 15) == 0) {
            uint4 *q = static_cast<uint4 *>(z.p[r]);
            const size_t n4 = z.n[r] / 16;
            for (size_t i = t; i < n4; i += stride) q[i] = make_uint4(0u, 0u, 0u, 0u);
            const size_t tail = (z.n[r] - n4 * 16) / 4;
            if (t < tail) reinterpret_cast<unsigned *>(q + n4)[t] = 0u;
        } else {
            unsigned *q = static_cast<unsigned *>(z.p[r]);
            for (size_t i = t; i < z.n[r] / 4; i += stride) q[i] = 0u;
        }
    }
}
static int zero_regions(std::initializer_list<std::pair<void *, size_t>> regs, hipStream_t st)
{
    ZeroArgs z{};
    size_t tot = 0;
    auto flush = [&]() -> int {
        if (!z.nr) return 0;
        const size_t blocks = std::min<size_t>(2048, std::max<size_t>(1, (tot / 16 + 255) / 256));
        hipLaunchKernelGGL(k_zero_regions, dim3((unsigned)blocks), dim3(256), 0, st, z);
        RDQ_CHECK(hipGetLastError());
        z = ZeroArgs{};
        tot = 0;
        return 0;
    };
    for (const auto &r : regs)                   // every region is 4-byte words: checked before any launch
        if (r.first && (r.second & 3)) return RDQ_E_INVALID;
    for (const auto &r : regs) {
        if (!r.first || !r.second) continue;
        if (z.nr == ZERO_MAXR) RDQ_TRY(flush());
        z.p[z.nr] = r.first;
        z.n[z.nr++] = r.second;
        tot += r.second;
    }
    return flush();
}

int launch_forward_pt(rdq_fwi_plan *p, int B, int NW, int per, const float *coeffs, float *seis, float *hist, float *ring,
                      hipStream_t st)
{
    FwdPtArgs a{};
    a.g = tb_geo(p, B);
    const int T = p->fwd_T;
    const size_t L = a.g.level;
    // granules, the history's first two slots and the first group's arrival counters: one launch
    if (int e = zero_regions({{hist, hist ? 2 * L * sizeof(float) : 0}, {ring, 4 * L * sizeof(unsigned long long)},
                              {p->d_status + 16, 8 * sizeof(unsigned)}}, st))
        return e;
    const int ih = region_rows(NW) - 4 * T;
    a.g.tiles_x = tiles_x(p->Wp, T);
    a.g.ntiles = a.g.tiles_x * ((p->Hp + ih - 1) / ih);
    a.coeffs = coeffs; a.wav = p->d_wav; a.hist = hist; a.seis = seis;
    a.gran = reinterpret_cast<unsigned long long *>(ring);
    a.status = p->d_status; a.nt = p->g.nt; a.prof = p->d_prof; a.xcd_mode = p->xcd_mode;
    a.sweep_delay = p->fwd_delay;
    // consecutive slice groups, one resident launch each (granules live at per-slice offsets, so
    // one zeroing serves every group)
    for (int s0 = 0; s0 < B * p->g.ns; s0 += per) {
        a.g.sl_off = s0;
        a.g.nsl = std::min(per, B * p->g.ns - s0);
        const dim3 grid(pt_grid(p, T, NW, a.g.nsl, false));
        if (s0 > 0) RDQ_TRY(zero_regions({{p->d_status + 16, 8 * sizeof(unsigned)}}, st));   // pt_assign arrivals
        launch_fwd_pt(p, NW, T, grid, st, a);
        RDQ_CHECK(hipGetLastError());
    }
    return 0;
}

int launch_adjoint_pt(rdq_fwi_plan *p, int B, int NW, int per, const float *coeffs, const float *hist, const float *dseis,
                      float *ring, float *gA, double *gk, float *gbeta, hipStream_t st)
{
    AdjPtArgs a{};
    a.g = tb_geo(p, B);
    const int T = p->adj_T;
    const size_t L = a.g.level;
    const int nblk_alloc = gk_blocks(p);
    if (int e = zero_regions({{ring, 4 * L * sizeof(unsigned long long)}, {gA, L * sizeof(float)},
                              {gk, (size_t)B * p->g.ns * nblk_alloc * sizeof(double)},
                              {gbeta, (size_t)B * p->g.ns * sizeof(float)}, {p->d_status + 16, 8 * sizeof(unsigned)}},
                             st))
        return e;
    const int ih = region_rows(NW) - 4 * T;
    a.g.tiles_x = tiles_x(p->Wp, T);
    a.g.ntiles = a.g.tiles_x * ((p->Hp + ih - 1) / ih);
    a.coeffs = coeffs; a.wav = p->d_wav; a.hist = hist; a.dseis = dseis;
    a.gA = gA; a.gk_part = gk; a.gbeta = gbeta;
    a.gran = reinterpret_cast<unsigned long long *>(ring);
    a.status = p->d_status; a.nt = p->g.nt; a.nblk = nblk_alloc; a.prof = p->d_prof ? p->d_prof + PROF_WORDS : nullptr;
    a.xcd_mode = p->xcd_mode;
    a.sweep_delay = p->adj_delay;
    for (int s0 = 0; s0 < B * p->g.ns; s0 += per) {
        a.g.sl_off = s0;
        a.g.nsl = std::min(per, B * p->g.ns - s0);
        const dim3 grid(pt_grid(p, T, NW, a.g.nsl, true));
        if (s0 > 0) RDQ_TRY(zero_regions({{p->d_status + 16, 8 * sizeof(unsigned)}}, st));   // pt_assign arrivals
        launch_adj_pt(p, NW, T, grid, st, a);
        RDQ_CHECK(hipGetLastError());
    }
    return 0;
}

int launch_forward(rdq_fwi_plan *p, int B, const float *coeffs, float *seis, float *hist,
                   float *ring, hipStream_t st)
{
    FwdTBArgs a{};
    a.g = tb_geo(p, B);
    const size_t L = a.g.level;
    const int T = p->wide ? wide_fwd_depth(p) : p->fwd_T, S = chain_count(p), ns = p->g.ns;
    // (no hipMemsetAsync under graph capture: see zero_regions)
    if (hist) RDQ_TRY(zero_regions({{hist, 2 * L * sizeof(float)}}, st));
    else RDQ_TRY(zero_regions({{ring, 4 * L * sizeof(float)}}, st));
    a.coeffs = coeffs;
    a.cg = coef_gen(p, B, coeffs);
    a.seis = seis;
    a.hist = hist;
    RDQ_TRY(fork_chains(p, st, S));
    const int nt = p->g.nt;
    for (int c = 0; c < S; ++c) {
        a.g.s_off = c * ns / S;
        a.g.ns_grp = (c + 1) * ns / S - a.g.s_off;
        a.ns_sh = a.g.ns_grp;            // wide kernels: a.spw shots of one region per workgroup
        const hipStream_t cs = c == 0 ? st : p->aux[c - 1];
        for (int n0 = 0, i = 0; n0 < nt; n0 += T, ++i) {
            a.n0 = n0;
            a.nsteps = std::min(T, nt - n0);
            // tile grid of this launch's depth (the wide kernels run a short tail as its own T)
            const int Tl = p->wide ? a.nsteps : T;
            a.g.tiles_x = p->wide ? tw_tiles_x(p->Wp, Tl) : tiles_x(p->Wp, Tl);
            a.g.ntiles = a.g.tiles_x * (p->wide ? tw_tiles_y(p->Hp, Tl, false) : tiles_y(p->Hp, Tl));
            a.spw = p->wide ? wide_spw(p->fwd_spw, B * a.g.ntiles, a.ns_sh, false, S) : 1;
            a.g.ns_grp = (a.ns_sh + a.spw - 1) / a.spw;
            const dim3 grid((a.g.ntiles + 7) / 8 * 8 * B * a.g.ns_grp);
            for (int t = 0; t < FWD_W_MAX; ++t) a.w[t] = t < a.nsteps ? p->wavf[n0 + t] : 0.0f;
            if (hist) {
                a.in_prev = hist + (size_t)n0 * L;          // slot n0   = P_{n0-1}
                a.in_cur = hist + (size_t)(n0 + 1) * L;     // slot n0+1 = P_{n0}
                a.out_prev = a.out_cur = nullptr;
            } else {
                const int pin = i & 1, pout = pin ^ 1;
                a.in_prev = ring + (size_t)(2 * pin) * L;
                a.in_cur = ring + (size_t)(2 * pin + 1) * L;
                a.out_prev = ring + (size_t)(2 * pout) * L;
                a.out_cur = ring + (size_t)(2 * pout + 1) * L;
            }
            if (p->wide) launch_fwd_w(a.nsteps, p->fwd_gen, (p->Wp & 1) == 0, grid, cs, a);   // (tail: T' < T)
            else launch_fwd(T, p->fwd_gen, grid, cs, a);
        }
    }
    RDQ_CHECK(hipGetLastError());
    return join_chains(p, st, S);
}

int launch_adjoint(rdq_fwi_plan *p, int B, const float *coeffs, const float *hist,
                   const float *dseis, float *ring, float *gA, double *gk, float *gbeta, hipStream_t st)
{
    AdjTBArgs a{};
    a.g = tb_geo(p, B);
    const size_t L = a.g.level;
    const int T = p->wide ? wide_adj_depth(p) : p->adj_T, S = chain_count(p), ns = p->g.ns;
    const int nblk_alloc = gk_blocks(p);
    a.coeffs = coeffs; a.hist = hist; a.dseis = dseis; a.gA = gA; a.gk_part = gk; a.gbeta = gbeta;
    a.cg = coef_gen(p, B, coeffs);
    a.nblk = nblk_alloc;
    // launch geometry of chain c's launch of depth nsteps: sets a.g.{s_off, tiles_x, ntiles, ns_grp},
    // a.ns_sh, a.spw; returns the grid size
    auto geometry = [&](int c, int nsteps) -> unsigned {
        a.g.s_off = c * ns / S;
        a.ns_sh = (c + 1) * ns / S - a.g.s_off;   // wide kernels: a.spw shots of one region per workgroup
        const int Tl = p->wide ? nsteps : T;
        a.g.tiles_x = p->wide ? tw_tiles_x(p->Wp, Tl) : tiles_x(p->Wp, Tl);
        a.g.ntiles = a.g.tiles_x * (p->wide ? tw_tiles_y(p->Hp, Tl, true) : tiles_y(p->Hp, Tl));
        a.spw = p->wide ? wide_spw(p->adj_spw, B * a.g.ntiles, a.ns_sh, true, S) : 1;
        a.g.ns_grp = (a.ns_sh + a.spw - 1) / a.spw;   // (the decode's slice groups are shot groups)
        return (unsigned)((a.g.ntiles + 7) / 8 * 8 * B * a.g.ns_grp);
    };
    {   // the gk_part one-writer invariant, on every launch, before anything is enqueued
        GkWriters writers((size_t)B * ns, nblk_alloc);
        for (int c = 0; c < S; ++c)
            for (int k0 = p->g.nt; k0 >= 1; k0 -= T) {
                const unsigned grid = geometry(c, std::min(T, k0));
                if (!writers.add(c, grid, a.g.tiles_x, a.g.ntiles, B, ns, a.g.ns_grp, a.g.s_off, a.spw, a.ns_sh))
                    return RDQ_E_INVALID;
            }
    }
    RDQ_TRY(zero_regions({{ring, 4 * L * sizeof(float)}, {gA, L * sizeof(float)},
                          {gk, (size_t)B * ns * nblk_alloc * sizeof(double)}, {gbeta, (size_t)B * ns * sizeof(float)}},
                         st));   // (no hipMemsetAsync under graph capture: see zero_regions)
    RDQ_TRY(fork_chains(p, st, S));
    for (int c = 0; c < S; ++c) {
        const hipStream_t cs = c == 0 ? st : p->aux[c - 1];
        for (int k0 = p->g.nt, i = 0; k0 >= 1; k0 -= T, ++i) {
            a.k0 = k0;
            a.nsteps = std::min(T, k0);
            const dim3 grid(geometry(c, a.nsteps));
            for (int t = 0; t < ADJ_W_MAX; ++t) a.w[t] = t < a.nsteps ? p->wavf[k0 - 1 - t] : 0.0f;
            const int pin = i & 1, pout = pin ^ 1;
            a.in_l1 = ring + (size_t)(2 * pin) * L;
            a.in_l2 = ring + (size_t)(2 * pin + 1) * L;
            a.out_l1 = ring + (size_t)(2 * pout) * L;
            a.out_l2 = ring + (size_t)(2 * pout + 1) * L;
            // (tail: T' < T); the exact order unless RDQ_VARIANT_CHUNKED_ADJ_FMA asked for the contracted
            // stencils (and only where nbc >= 20: a thin sponge's standing modes amplify the contraction)
            if (p->wide) launch_adj_w(a.nsteps, (p->Wp & 1) == 0, !p->adj_tw_fma, grid, cs, a);
            else launch_adj(T, grid, cs, a);
        }
    }
    RDQ_CHECK(hipGetLastError());
    return join_chains(p, st, S);
}

// destroy every cached graph; a graph may still be queued or running (asynchronous launches), so
// the device is drained first
void drop_graphs(rdq_fwi_plan *p)
{
    if (p->cache.empty()) return;
    (void)hipDeviceSynchronize();
    for (auto &e : p->cache) (void)hipGraphExecDestroy(e.exec);
    p->cache.clear();
}

template <class F>
int run_cached(rdq_fwi_plan *p, int kind, int B, std::initializer_list<const void *> key, hipStream_t st, F &&launch)
{
    if (!p->graphs) return launch(st);
    const void *k[8] = {nullptr};
    int n = 0;
    for (const void *v : key) k[n++] = v;
    for (auto &e : p->cache)
        if (e.kind == kind && e.B == B && std::equal(k, k + 8, e.ptrs)) {
            e.last_use = ++p->tick;
            RDQ_CHECK(hipGraphLaunch(e.exec, st));
            return 0;
        }
    if (!p->cap) RDQ_CHECK(hipStreamCreateWithFlags(&p->cap, hipStreamNonBlocking));
    hipGraph_t graph = nullptr;
    RDQ_CHECK(hipStreamBeginCapture(p->cap, hipStreamCaptureModeThreadLocal));
    const int rc = launch(p->cap);
    const hipError_t ee = hipStreamEndCapture(p->cap, &graph);
    if (rc) { if (graph) (void)hipGraphDestroy(graph); return rc; }
    RDQ_CHECK(ee);
    GraphEntry e{};
    e.kind = kind; e.B = B;
    std::copy(k, k + 8, e.ptrs);
    const hipError_t ie = hipGraphInstantiate(&e.exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    RDQ_CHECK(ie);
    e.last_use = ++p->tick;
    if (p->cache.size() >= 16) {
        auto old = std::min_element(p->cache.begin(), p->cache.end(),
                                    [](const GraphEntry &a, const GraphEntry &b) { return a.last_use < b.last_use; });
        // the evicted graph may still be queued or running on `st` (everything here is
        // asynchronous): destroying an executing graph frees its kernel-argument storage under the
        // running persistent kernel, so drain the stream first (evictions are rare: a steady loop
        // replays cached graphs)
        RDQ_CHECK(hipStreamSynchronize(st));
        (void)hipGraphExecDestroy(old->exec);
        p->cache.erase(old);
    }
    p->cache.push_back(e);
    RDQ_CHECK(hipGraphLaunch(e.exec, st));
    return 0;
}

}  // namespace

// ======================================================================================= C ABI
extern "C" {

// The recurrence adjoint (k_adj_pr) recovers lap'(P_{k-1}) = (P_k - T1 P_{k-1} + T2 P_{k-2} - src) / A
// from three history levels: a difference of nearly equal values whenever the field is smooth on
// the grid scale.  With an absorbing sponge (the reference's nbc = 120) the field keeps its
// wavelength and the gradient stays within ~1e-5 of the exact order (profiles/r3/
// small_dt_adjoint.jsonl: 1.0e-5 at dt = 1 ms, 3.9e-5 at dt / 4); a thin sponge lets the wave wrap
// round the periodic grid into long standing modes and the cancellation costs 5e-3 (tests/
// golden/fwd_wrap: nbc = 4).  Below RDQ_RECURRENCE_MIN_NBC the plan runs the exact-order adjoint.
constexpr int RDQ_RECURRENCE_MIN_NBC = 20;
static bool recurrence_ok(const rdq_fwi_plan *p) { return p->g.nbc >= RDQ_RECURRENCE_MIN_NBC; }

int rdq_fwi_plan_create(const rdq_fwi_geom *geom, rdq_fwi_plan **out)
{
    if (!geom || !out || geom->nz < 1 || geom->nx < 1 || geom->nbc < 0 || geom->nt < 1 || geom->ns < 1 ||
        geom->ng < 1 || geom->sample_temporal < 1 || !geom->isx || !geom->igx || !geom->wavelet)
        return RDQ_E_INVALID;
    rdq_fwi_plan *p = new (std::nothrow) rdq_fwi_plan();
    if (!p) return RDQ_E_NOMEM;
    p->g = *geom;
    p->Hp = geom->nz + 2 * geom->nbc;
    p->Wp = geom->nx + 2 * geom->nbc;
    p->ld = (p->Wp + 63) / 64 * 64;
    p->nrec = (geom->nt + geom->sample_temporal - 1) / geom->sample_temporal;
    p->isx.assign(geom->isx, geom->isx + geom->ns);
    p->igx.assign(geom->igx, geom->igx + geom->ng);
    p->wav.assign(geom->wavelet, geom->wavelet + geom->nt);
    p->wavf.resize(geom->nt);
    for (int i = 0; i < geom->nt; ++i) p->wavf[i] = (float)p->wav[i];   // pde.py:81 casts to fp32
    for (int v : p->isx) if (v < 0 || v >= p->Wp) { delete p; return RDQ_E_INVALID; }
    for (int v : p->igx) if (v < 0 || v >= p->Wp) { delete p; return RDQ_E_INVALID; }
    if (geom->isz < 0 || geom->isz >= p->Hp || geom->igz < 0 || geom->igz >= p->Hp) { delete p; return RDQ_E_INVALID; }
    if (p->Wp > FIN_MAXW) { delete p; return RDQ_E_INVALID; }   // gradient finalize holds a padded row in LDS
    p->g.isx = p->isx.data();
    p->g.igx = p->igx.data();
    p->g.wavelet = p->wav.data();
    // receivers grouped by column (stable -> ascending receiver id within a column)
    std::vector<int> order(geom->ng), start(p->Wp + 1, 0);
    for (int r = 0; r < geom->ng; ++r) order[r] = r;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return p->igx[a] < p->igx[b]; });
    for (int r = 0; r < geom->ng; ++r) start[p->igx[r] + 1]++;
    for (int x = 0; x < p->Wp; ++x) start[x + 1] += start[x];
    // adjoint residual per column: the receiver's own dseis, or (several receivers in one column)
    // their residuals folded in receiver order into one value per column (k_rcv_fold)
    std::vector<int> rlane(p->Wp, -1), colx;
    for (int x = 0; x < p->Wp; ++x) {
        if (start[x + 1] - start[x] > 1) p->rmulti = true;
        if (start[x + 1] > start[x]) colx.push_back(x);
    }
    p->ncolr = (int)colx.size();
    for (int c = 0; c < p->ncolr; ++c) rlane[colx[c]] = p->rmulti ? c : order[start[colx[c]]];
    hipError_t e = hipMalloc(&p->d_isx, sizeof(int) * geom->ns);
    if (e == hipSuccess) e = hipMalloc(&p->d_rcv_start, sizeof(int) * (p->Wp + 1));
    if (e == hipSuccess) e = hipMalloc(&p->d_rcv_list, sizeof(int) * geom->ng);
    if (e == hipSuccess) e = hipMemcpy(p->d_isx, p->isx.data(), sizeof(int) * geom->ns, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(p->d_rcv_start, start.data(), sizeof(int) * (p->Wp + 1), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(p->d_rcv_list, order.data(), sizeof(int) * geom->ng, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&p->d_rlane, sizeof(int) * p->Wp);
    if (e == hipSuccess) e = hipMemcpy(p->d_rlane, rlane.data(), sizeof(int) * p->Wp, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&p->d_colx, sizeof(int) * std::max(p->ncolr, 1));
    if (e == hipSuccess && p->ncolr)
        e = hipMemcpy(p->d_colx, colx.data(), sizeof(int) * p->ncolr, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&p->d_wav, sizeof(float) * geom->nt);
    if (e == hipSuccess) e = hipMemcpy(p->d_wav, p->wavf.data(), sizeof(float) * geom->nt, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&p->d_status_own, 256);
    if (e == hipSuccess) e = hipMemset(p->d_status_own, 0, 256);
    p->d_status = p->d_status_own;
    p->adj_fma = recurrence_ok(p);
    if (e != hipSuccess) { rdq_fwi_plan_destroy(p); return -(int)e; }
    *out = p;
    return 0;
}

int rdq_fwi_plan_destroy(rdq_fwi_plan *p)
{
    if (!p) return 0;
    drop_graphs(p);
    if (p->cap) (void)hipStreamDestroy(p->cap);
    for (auto st : p->aux) (void)hipStreamDestroy(st);
    for (auto e : p->evs) (void)hipEventDestroy(e);
    if (p->handover) (void)hipEventDestroy(p->handover);
    if (p->d_isx) (void)hipFree(p->d_isx);
    if (p->d_rcv_start) (void)hipFree(p->d_rcv_start);
    if (p->d_rcv_list) (void)hipFree(p->d_rcv_list);
    if (p->d_rlane) (void)hipFree(p->d_rlane);
    if (p->d_colx) (void)hipFree(p->d_colx);
    if (p->d_wav) (void)hipFree(p->d_wav);
    if (p->d_status_own) (void)hipFree(p->d_status_own);
    if (p->d_prof) (void)hipFree(p->d_prof);
    delete p;
    return 0;
}

int rdq_fwi_set_graphs(rdq_fwi_plan *p, int32_t enable)
{
    if (!p) return RDQ_E_INVALID;
    std::lock_guard<std::mutex> lk(p->mu);
    p->graphs = enable != 0;
    return 0;
}

int rdq_fwi_set_tuning(rdq_fwi_plan *p, int32_t fwd_steps, int32_t adj_steps, int32_t chains)
{
    if (!p || fwd_steps < 1 || fwd_steps > TB_MAXT || adj_steps < 1 || adj_steps > TB_MAXT || chains < 0 ||
        chains > 16)
        return RDQ_E_INVALID;
    std::lock_guard<std::mutex> lk(p->mu);
    if (p->fwd_T != fwd_steps || p->adj_T != adj_steps || p->chains != chains) {   // graphs encode these
        drop_graphs(p);
        p->cache.clear();
    }
    p->fwd_T = fwd_steps;
    p->adj_T = adj_steps;
    p->chains = chains;
    return 0;
}

int rdq_fwi_set_wide_fwd_steps(rdq_fwi_plan *p, int32_t steps)
{
    if (!p || steps < 0 || steps > TW_FWD_MAXT) return RDQ_E_INVALID;   // 0 = set_tuning's fwd_steps
    std::lock_guard<std::mutex> lk(p->mu);
    if (p->fwd_Tw != steps) {   // graphs encode the launch sequence
        drop_graphs(p);
        p->cache.clear();
    }
    p->fwd_Tw = steps;
    return 0;
}

int rdq_fwi_set_wide_fwd_shots(rdq_fwi_plan *p, int32_t shots)
{
    if (!p || shots < 0 || shots > 64) return RDQ_E_INVALID;   // 0 = auto (wide_spw)
    std::lock_guard<std::mutex> lk(p->mu);
    if (p->fwd_spw != shots) {   // graphs encode the grids
        drop_graphs(p);
        p->cache.clear();
    }
    p->fwd_spw = shots;
    return 0;
}

int rdq_fwi_set_wide_adj_shots(rdq_fwi_plan *p, int32_t shots)
{
    if (!p || shots < 0 || shots > 64) return RDQ_E_INVALID;   // 0 = auto (wide_spw)
    std::lock_guard<std::mutex> lk(p->mu);
    if (p->adj_spw != shots) {   // graphs encode the grids
        drop_graphs(p);
        p->cache.clear();
    }
    p->adj_spw = shots;
    return 0;
}

int rdq_fwi_set_wide_adj_steps(rdq_fwi_plan *p, int32_t steps)
{
    if (!p || steps < 0 || steps > TW_ADJ_MAXT) return RDQ_E_INVALID;   // 0 = auto (wide_adj_depth)
    std::lock_guard<std::mutex> lk(p->mu);
    if (wide_adj_depth(p) != (steps ? steps : TW_ADJ_DEFAULT)) {   // graphs encode the launch sequence
        drop_graphs(p);
        p->cache.clear();
    }
    p->adj_Tw = steps;
    return 0;
}

int rdq_fwi_set_variant(rdq_fwi_plan *p, int32_t flags)
{
    if (!p || (flags & ~31)) return RDQ_E_INVALID;
    std::lock_guard<std::mutex> lk(p->mu);
    const bool gen = (flags & RDQ_VARIANT_FWD_GEN) != 0;
    const bool fma = (flags & RDQ_VARIANT_ADJ_EXACT) == 0 && recurrence_ok(p);
    const bool twfma = (flags & RDQ_VARIANT_CHUNKED_ADJ_FMA) != 0 && (flags & RDQ_VARIANT_ADJ_EXACT) == 0 &&
                       recurrence_ok(p);
    const int xcd = (flags & RDQ_VARIANT_NO_XCD_LOCAL) ? 0 : 1;
    const bool wide = (flags & RDQ_VARIANT_NARROW_CHUNKED) == 0;
    if (p->fwd_gen != gen || p->adj_fma != fma || p->adj_tw_fma != twfma || p->xcd_mode != xcd || p->wide != wide) {
        drop_graphs(p);
        p->cache.clear();
    }
    p->fwd_gen = gen;
    p->adj_fma = fma;
    p->adj_tw_fma = twfma;
    p->xcd_mode = xcd;
    p->wide = wide;
    return 0;
}

int rdq_fwi_set_rows_per_wave(rdq_fwi_plan *p, int32_t fwd_rows, int32_t adj_rows)
{
    if (!p || (fwd_rows != 6 && fwd_rows != 8 && fwd_rows != 12 && fwd_rows != 24) ||
        (adj_rows != 6 && adj_rows != 8 && adj_rows != 12))
        return RDQ_E_INVALID;
    std::lock_guard<std::mutex> lk(p->mu);
    if (p->fwd_rw != fwd_rows || p->adj_rw != adj_rows) {
        drop_graphs(p);
        p->cache.clear();
    }
    p->fwd_rw = fwd_rows;
    p->adj_rw = adj_rows;
    return 0;
}
int rdq_fwi_set_persistent(rdq_fwi_plan *p, int32_t mode)
{
    if (!p || (mode != 0 && mode != 1 && mode != 8 && mode != 12 && mode != 16 && mode != -1)) return RDQ_E_INVALID;
    std::lock_guard<std::mutex> lk(p->mu);
    if (p->persist != mode) {
        drop_graphs(p);
        p->cache.clear();
    }
    p->persist = mode;
    return 0;
}

int rdq_fwi_launch_info(rdq_fwi_plan *p, int32_t B, int32_t out[6])
{
    if (!p || !out || B < 1) return RDQ_E_INVALID;
    std::lock_guard<std::mutex> lk(p->mu);
    int perf = 0, pera = 0;
    out[0] = persistent_nw(p, B, false, &perf);
    out[1] = persistent_nw(p, B, true, &pera);
    const int fwdT = !out[0] && p->wide ? wide_fwd_depth(p) : p->fwd_T;   // chunked forward: the wide kernels' depth
    out[2] = fwdT;
    const int adjT = !out[1] && p->wide ? wide_adj_depth(p) : p->adj_T;   // chunked adjoint: the wide kernels' depth
    out[3] = adjT;
    const int ns = B * p->g.ns, nt = p->g.nt;   // persistent: one launch per slice group
    out[4] = out[0] ? (ns + perf - 1) / perf : (nt + fwdT - 1) / fwdT;
    out[5] = out[1] ? (ns + pera - 1) / pera : (nt + adjT - 1) / adjT;
    return 0;
}

int rdq_fwi_set_sweep_delay(rdq_fwi_plan *p, int32_t fwd_ticks, int32_t adj_ticks)
{
    if (!p || fwd_ticks < 0 || fwd_ticks > 100000 || adj_ticks < 0 || adj_ticks > 100000) return RDQ_E_INVALID;
    std::lock_guard<std::mutex> lk(p->mu);
    p->fwd_delay = fwd_ticks;   // (persistent launches are direct, not graphs: nothing cached to drop)
    p->adj_delay = adj_ticks;
    return 0;
}

int rdq_fwi_wide_info(rdq_fwi_plan *p, int32_t B, int32_t out[4])
{
    if (!p || !out || B < 1) return RDQ_E_INVALID;
    std::lock_guard<std::mutex> lk(p->mu);
    const int S = chain_count(p), ns0 = p->g.ns / S;   // chain 0: shots [0, ns / S), the smallest group
    const int Tf = wide_fwd_depth(p), Ta = wide_adj_depth(p);
    out[0] = S;
    out[1] = p->wide ? wide_spw(p->fwd_spw, B * tw_tiles_x(p->Wp, Tf) * tw_tiles_y(p->Hp, Tf, false), ns0, false, S) : 1;
    out[2] = p->wide ? wide_spw(p->adj_spw, B * tw_tiles_x(p->Wp, Ta) * tw_tiles_y(p->Hp, Ta, true), ns0, true, S) : 1;
    out[3] = ns0;
    return 0;
}

int rdq_fwi_set_profile(rdq_fwi_plan *p, int32_t enable)
{
    if (!p) return RDQ_E_INVALID;
    std::lock_guard<std::mutex> lk(p->mu);
    drop_graphs(p);   // graphs bake the pointer in
    p->cache.clear();
    if (enable && !p->d_prof) {
        RDQ_CHECK(hipMalloc(&p->d_prof, 2 * PROF_WORDS * sizeof(unsigned long long)));
        RDQ_CHECK(hipMemset(p->d_prof, 0, 2 * PROF_WORDS * sizeof(unsigned long long)));
    } else if (!enable && p->d_prof) {
        RDQ_CHECK(hipFree(p->d_prof));
        p->d_prof = nullptr;
    }
    return 0;
}

int rdq_fwi_read_profile(rdq_fwi_plan *p, uint64_t out[12])
{
    if (!p || !out) return RDQ_E_INVALID;
    std::lock_guard<std::mutex> lk(p->mu);
    if (!p->d_prof) { for (int i = 0; i < 8; ++i) out[i] = 0; return 0; }
    RDQ_CHECK(hipDeviceSynchronize());
    p->prof_host.resize(2 * PROF_WORDS);
    RDQ_CHECK(hipMemcpy(p->prof_host.data(), p->d_prof, 2 * PROF_WORDS * sizeof(unsigned long long),
                        hipMemcpyDeviceToHost));
    RDQ_CHECK(hipMemset(p->d_prof, 0, 2 * PROF_WORDS * sizeof(unsigned long long)));
    for (int i = 0; i < 6; ++i) { out[i] = p->prof_host[i]; out[6 + i] = p->prof_host[PROF_WORDS + i]; }
    return 0;
}

int rdq_fwi_profile_waves(rdq_fwi_plan *p, int32_t adj, uint64_t *out, size_t count)
{
    if (!p || !out || (adj != 0 && adj != 1)) return RDQ_E_INVALID;
    std::lock_guard<std::mutex> lk(p->mu);
    const size_t n = std::min(count, PROF_WAVES * 3);
    for (size_t i = 0; i < n; ++i)
        out[i] = p->prof_host.empty() ? 0 : p->prof_host[(adj ? PROF_WORDS : 0) + PROF_RAW + i];
    return 0;
}

int rdq_fwi_status(rdq_fwi_plan *p, hipStream_t st)
{
    if (!p) return RDQ_E_INVALID;
    std::lock_guard<std::mutex> lk(p->mu);
    unsigned v = 0;
    RDQ_CHECK(hipMemcpyAsync(&v, p->d_status, sizeof(v), hipMemcpyDeviceToHost, st));
    RDQ_CHECK(hipStreamSynchronize(st));
    if (v) {
        RDQ_CHECK(hipMemsetAsync(p->d_status, 0, sizeof(v), st));
        RDQ_CHECK(hipStreamSynchronize(st));
        return RDQ_E_HANDOFF;
    }
    return 0;
}

int rdq_fwi_set_status_buffer(rdq_fwi_plan *p, uint32_t *words)
{
    if (!p) return RDQ_E_INVALID;
    std::lock_guard<std::mutex> lk(p->mu);
    if (p->d_status != (words ? words : p->d_status_own)) {
        drop_graphs(p);
        p->cache.clear();
    }
    p->d_status = words ? words : p->d_status_own;
    return 0;
}

int rdq_fwi_debug_words(rdq_fwi_plan *p, uint32_t out[32])
{
    if (!p || !out) return RDQ_E_INVALID;
    std::lock_guard<std::mutex> lk(p->mu);
    RDQ_CHECK(hipDeviceSynchronize());
    RDQ_CHECK(hipMemcpy(out, p->d_status, 32 * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return 0;
}

int rdq_fwi_sizes(const rdq_fwi_plan *p, int32_t B, rdq_fwi_sizes_t *o)
{
    if (!p || !o || B < 1) return RDQ_E_INVALID;
    const size_t slice = (size_t)p->Hp * p->ld, ns = p->g.ns;
    o->Hp = p->Hp; o->Wp = p->Wp; o->ld = p->ld; o->nrec = p->nrec;
    o->coeffs = (6 * (size_t)B * slice + (size_t)B * p->g.nz * p->g.nx + B + 4) * sizeof(float);
    o->vstat = (size_t)B * (sizeof(float) + sizeof(int64_t)) + 16;
    o->seis = (size_t)B * ns * p->nrec * p->g.ng * sizeof(float);
    o->history = (size_t)(p->g.nt + 2) * B * ns * slice * sizeof(float);
    o->ring = 4 * (size_t)B * ns * slice * sizeof(unsigned long long);
    if (p->rmulti) o->ring += (size_t)B * ns * p->nrec * p->ncolr * sizeof(float);   // folded residuals
    o->gA = (size_t)B * ns * slice * sizeof(float);
    o->gk_part = (size_t)B * ns * gk_blocks(p) * sizeof(double);
    o->gbeta = (size_t)B * ns * sizeof(float);
    o->colsum = (size_t)B * p->Hp * p->g.nx * sizeof(double);
    return 0;
}

static void vstat_ptrs(const void *vstat, int B, float **vmin, int64_t **amin)
{
    char *base = (char *)vstat;
    *vmin = (float *)base;
    *amin = (int64_t *)(base + (((size_t)B * sizeof(float) + 15) / 16) * 16);
}

int rdq_fwi_coeffs(const rdq_fwi_plan *p, int32_t B, const float *vn, const int64_t strides[4],
                   int32_t vel_mode, float *coeffs, void *vstat, hipStream_t st)
{
    if (!p || !vn || !strides || !coeffs || !vstat || B < 1 || (vel_mode != 0 && vel_mode != 1))
        return RDQ_E_INVALID;
    float *vmin; int64_t *amin;
    vstat_ptrs(vstat, B, &vmin, &amin);
    CoefArgs a;
    a.cg = coef_gen(p, B, coeffs);
    const double ad = (double)(p->g.nbc - 1) * (double)p->g.dx;   // a = (nbc-1)*dx, pde.py:42
    {   // partials in field 5 of `coeffs` (the model copy, written by k_coeff_fields afterwards)
        const int n = p->g.nz * p->g.nx, parts = std::max(1, std::min(256, (n + 8191) / 8192));
        const int chunk = (n + parts - 1) / parts;
        float *pv = coeffs + 5 * (size_t)B * p->Hp * p->ld;
        int64_t *pi = reinterpret_cast<int64_t *>(pv + (((size_t)B * parts + 3) / 4) * 4);
        hipLaunchKernelGGL(k_vstat_part, dim3(B, parts), dim3(256), 0, st, vn, strides[0], strides[2], strides[3],
                           p->g.nz, p->g.nx, vel_mode, chunk, pv, pi);
        hipLaunchKernelGGL(k_vstat_final, dim3(B), dim3(256), 0, st, pv, pi, parts, (float)std::log(10000000.0),
                           (float)(2.0 * ad), vmin, amin, const_cast<float *>(a.cg.ks));
    }
    a.vn = vn; a.s0 = strides[0]; a.s2 = strides[2]; a.s3 = strides[3];
    a.vel_mode = vel_mode; a.ld = p->ld;
    a.vmod_out = const_cast<float *>(a.cg.vmod);
    a.coeffs = coeffs;
    a.cstride = (size_t)B * p->Hp * p->ld;
    hipLaunchKernelGGL(k_coeffs, dim3((p->ld + 255) / 256, p->Hp, B), dim3(256), 0, st, a);
    hipLaunchKernelGGL(k_coeff_fields, dim3((p->ld + 255) / 256, p->Hp, B), dim3(256), 0, st, a);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

int rdq_fwi_forward(const rdq_fwi_plan *pc, int32_t B, const float *coeffs, float *seis, float *hist,
                    float *ring, hipStream_t st)
{
    rdq_fwi_plan *p = const_cast<rdq_fwi_plan *>(pc);
    if (!p || !coeffs || !seis || (!hist && !ring) || B < 1) return RDQ_E_INVALID;
    std::lock_guard<std::mutex> lk(p->mu);
    RDQ_TRY(plan_enter(p, st));
    int per = 0;
    if (const int nw = persistent_nw(p, B, false, &per)) {
        if (!ring) return RDQ_E_INVALID;   // the persistent kernel's hand-off granules live in `ring`
        // direct launch (one kernel + memsets per shot group: nothing for a graph to amortise; the
        // arrival counters of pt_assign are zeroed by a stream-ordered memset right before it)
        return launch_forward_pt(p, B, nw, per, coeffs, seis, hist, ring, st);
    }
    return run_cached(p, hist ? 0 : 1, B, {coeffs, seis, hist, ring}, st,
                      [&](hipStream_t s) { return launch_forward(p, B, coeffs, seis, hist, ring, s); });
}

int rdq_fwi_adjoint(const rdq_fwi_plan *pc, int32_t B, const float *coeffs, const float *hist,
                    const float *dseis, float *ring, float *gA, double *gk, float *gbeta, hipStream_t st)
{
    rdq_fwi_plan *p = const_cast<rdq_fwi_plan *>(pc);
    if (!p || !coeffs || !hist || !dseis || !ring || !gA || !gk || !gbeta || B < 1) return RDQ_E_INVALID;
    std::lock_guard<std::mutex> lk(p->mu);
    RDQ_TRY(plan_enter(p, st));
    if (p->rmulti) {   // several receivers in a column: fold the residuals per column (ring tail)
        float *fold = ring + 8 * (size_t)B * p->g.ns * p->Hp * p->ld;
        const size_t rows = (size_t)B * p->g.ns * p->nrec, n = rows * p->ncolr;
        hipLaunchKernelGGL(k_rcv_fold, dim3((unsigned)std::min<size_t>((n + 255) / 256, 4096)), dim3(256), 0, st,
                           dseis, fold, p->d_colx, p->d_rcv_start, p->d_rcv_list, p->g.ng, p->ncolr, rows);
        RDQ_CHECK(hipGetLastError());
        dseis = fold;
    }
    int per = 0;
    if (const int nw = persistent_nw(p, B, true, &per))
        return launch_adjoint_pt(p, B, nw, per, coeffs, hist, dseis, ring, gA, gk, gbeta, st);
    return run_cached(p, 2, B, {coeffs, hist, dseis, ring, gA, gk, gbeta}, st, [&](hipStream_t s) {
        return launch_adjoint(p, B, coeffs, hist, dseis, ring, gA, gk, gbeta, s);
    });
}

int rdq_fwi_grad_finalize(const rdq_fwi_plan *p, int32_t B, const float *coeffs, const void *vstat,
                          const float *gA, const double *gk, const float *gbeta, int32_t vel_mode,
                          double *colsum, float *out, hipStream_t st)
{
    if (!p || !coeffs || !vstat || !gA || !gk || !gbeta || !colsum || !out || B < 1 ||
        (vel_mode != 0 && vel_mode != 1))
        return RDQ_E_INVALID;
    float *vmin; int64_t *amin;
    vstat_ptrs(vstat, B, &vmin, &amin);
    FinArgs a;
    a.B = B; a.ns = p->g.ns; a.nz = p->g.nz; a.nx = p->g.nx; a.nbc = p->g.nbc; a.Hp = p->Hp; a.Wp = p->Wp;
    a.ld = p->ld; a.isz = p->g.isz; a.nblk = gk_blocks(p); a.dt = p->g.dt; a.dx = p->g.dx;
    a.scale = vel_mode == 0 ? 1500.0 : 1.0;
    a.slice = (size_t)p->Hp * p->ld; a.cstride = (size_t)B * a.slice;
    a.coeffs = coeffs; a.gA = gA; a.gbeta = gbeta; a.vmin = vmin; a.amin = amin; a.gk_part = gk;
    a.isx = p->d_isx; a.colsum = colsum; a.out = out;
    if (p->Wp > FIN_MAXW) return RDQ_E_INVALID;
    hipLaunchKernelGGL(k_fin_rows, dim3(p->Hp, B), dim3(256), 0, st, a);
    hipLaunchKernelGGL(k_fin_cols, dim3((p->g.nz * p->g.nx + 255) / 256, B), dim3(256), 0, st, a);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

size_t rdq_l1_partial_bytes(int32_t B, int64_t n)
{
    const int64_t nchunk = (n + L1_BLOCK * L1_ITEMS - 1) / (L1_BLOCK * L1_ITEMS);
    return (size_t)B * nchunk * 2 * sizeof(double);
}

int rdq_l1_forward(int32_t B, int64_t n, const float *pred, const float *y, const float *mask, float *loss,
                   float *nobs, void *partial, hipStream_t st)
{
    if (B < 1 || n < 1 || !pred || !y || !loss || !nobs || !partial) return RDQ_E_INVALID;
    const int nchunk = (int)((n + L1_BLOCK * L1_ITEMS - 1) / (L1_BLOCK * L1_ITEMS));
    hipLaunchKernelGGL(k_l1_partial, dim3(nchunk, B), dim3(L1_BLOCK), 0, st, n, pred, y, mask, (double *)partial, nchunk);
    hipLaunchKernelGGL(k_l1_final, dim3(B), dim3(L1_BLOCK), 0, st, B, nchunk, (const double *)partial, loss, nobs);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

int rdq_l1_backward(int32_t B, int64_t n, const float *pred, const float *y, const float *mask,
                    const float *nobs, const float *gout, float *dpred, hipStream_t st)
{
    if (B < 1 || n < 1 || !pred || !y || !nobs || !gout || !dpred) return RDQ_E_INVALID;
    hipLaunchKernelGGL(k_l1_backward, dim3((unsigned)((n + 255) / 256), B), dim3(256), 0, st, B, n, pred, y, mask,
                       nobs, gout, dpred);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

int rdq_smooth_reg_forward(int32_t kind, int32_t B, int32_t H, int32_t W, const float *mu, float *loss,
                           hipStream_t st)
{
    if ((kind != 0 && kind != 1) || B < 1 || H < 2 || W < 2 || !mu || !loss) return RDQ_E_INVALID;
    hipLaunchKernelGGL(k_smooth_fwd, dim3(B), dim3(256), 0, st, kind, H, W, mu, loss);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

int rdq_smooth_reg_backward(int32_t kind, int32_t B, int32_t H, int32_t W, const float *mu,
                            const float *gout, float *grad, hipStream_t st)
{
    if ((kind != 0 && kind != 1) || B < 1 || H < 2 || W < 2 || !mu || !gout || !grad) return RDQ_E_INVALID;
    hipLaunchKernelGGL(k_smooth_bwd, dim3((H * W + 255) / 256, B), dim3(256), 0, st, kind, H, W, mu, gout, grad);
    RDQ_CHECK(hipGetLastError());
    return 0;
}

}  // extern "C"
