/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the red-diffeq acoustic FWI hot path (forward propagator, discrete adjoint,
 * velocity gradient).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / the timed CPU baseline; the product path
 * (red-diffeq_amd/) never links or calls it.
 *
 * Reference being restated (all paths in SimingShan/red-diffeq):
 *   FWIForward.forward     red_diffeq/solvers/pde.py:88-93     denorm -> replicate pad -> FWM
 *   v_denormalize          red_diffeq/utils/data_trans.py:13-15 (v+1)/2*3000+1500
 *   get_Abc                red_diffeq/solvers/pde.py:38-52     sponge; columns overwrite rows
 *   FWM                    red_diffeq/solvers/pde.py:61-86     coefficient fields + time loop
 *   autograd backward      (no code; triggered red_diffeq/core/inversion.py:86) -> discrete
 *                          adjoint derived in SURVEY.md §3.5.
 *
 * Pinning: forward seismograms are compared BIT-FOR-BIT with fixtures produced by the reference
 * (tests/golden/make_golden.py); gradients within fp32 tolerance of the reference's autograd.
 * The fp32 operation order below follows the reference's PyTorch expression order exactly, and
 * this file must be compiled with -ffp-contract=off (no FMA contraction) for that to hold.
 *
 * Layout (dense, no padding): fields [B][Hp][Wp]; wavefields [B][ns][Hp][Wp];
 * seis [B][ns][nrec][ng]; history slot j holds P_{j-1} (slots 0,1 are zero), nt+2 slots of
 * [B][ns][Hp][Wp].
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    int B, ns, ng, nt, nz, nx, nbc, st; /* st = sample_temporal */
    float dx, dt;
    int isz, igz;
    const int *isx;       /* [ns] padded-grid column of each source */
    const int *igx;       /* [ng] padded-grid column of each receiver */
    const double *wavelet; /* [nt] Ricker wavelet, fp64 as the reference keeps it (pde.py:26-36) */
} oracle_geom;

static const float C1X2 = -5.0f;                 /* 2*c1, c1 = -2.5 (pde.py:66,69) */
static const float C2 = (float)(4.0 / 3.0);      /* pde.py:67 */
static const float C3 = (float)(-1.0 / 12.0);    /* pde.py:68 */

static inline int Hp_of(const oracle_geom *g) { return g->nz + 2 * g->nbc; }
static inline int Wp_of(const oracle_geom *g) { return g->nx + 2 * g->nbc; }
int oracle_nrec(const oracle_geom *g) { return (g->nt + g->st - 1) / g->st; }

/* v_denormalize (data_trans.py:13-15) then F.pad(replicate) (pde.py:91). */
void oracle_vpad(const oracle_geom *g, const float *vnorm, float *vpad)
{
    const int Hp = Hp_of(g), Wp = Wp_of(g);
    for (int b = 0; b < g->B; ++b)
        for (int z = 0; z < Hp; ++z) {
            int iz = z - g->nbc; iz = iz < 0 ? 0 : (iz >= g->nz ? g->nz - 1 : iz);
            for (int x = 0; x < Wp; ++x) {
                int ix = x - g->nbc; ix = ix < 0 ? 0 : (ix >= g->nx ? g->nx - 1 : ix);
                float t = vnorm[((size_t)b * g->nz + iz) * g->nx + ix];
                t = t + 1.0f; t = t / 2.0f; t = t * 3000.0f; t = t + 1500.0f;
                vpad[((size_t)b * Hp + z) * Wp + x] = t;
            }
        }
}

/* Sponge profile + coefficient fields (pde.py:38-52, 63-71).  argmin is the FIRST row-major
 * index of the minimum over the padded field (torch.min tie rule, pde.py:41). */
void oracle_coeffs(const oracle_geom *g, const float *vpad, float *alpha, float *temp1,
                   float *temp2, float *kappa, float *beta, float *vmin, int64_t *argmin)
{
    const int Hp = Hp_of(g), Wp = Wp_of(g), nbc = g->nbc;
    const float dt = g->dt, dx = g->dx;
    const float a = (float)((nbc - 1) * (double)dx);
    const float lnk = (float)log(10000000.0);
    float *prof = (float *)malloc(sizeof(float) * (nbc > 0 ? nbc : 1));
    for (int b = 0; b < g->B; ++b) {
        const float *v = vpad + (size_t)b * Hp * Wp;
        float m = v[0]; int64_t am = 0;
        for (int64_t i = 1; i < (int64_t)Hp * Wp; ++i) if (v[i] < m) { m = v[i]; am = i; }
        vmin[b] = m; argmin[b] = am;
        /* kappa = 3.0*velmin*np.log(1e7)/(2.0*a) */
        float ks = 3.0f * m; ks = ks * lnk; ks = ks / (float)(2.0 * (double)a);
        for (int i = 0; i < nbc; ++i) {
            float d = (float)i * dx; d = d / a; d = d * d; prof[i] = ks * d;  /* damp1d */
        }
        for (int z = 0; z < Hp; ++z)
            for (int x = 0; x < Wp; ++x) {
                float dmp = 0.0f;
                if (z < nbc) dmp = prof[nbc - 1 - z];
                if (z >= Hp - nbc) dmp = prof[z - (Hp - nbc)];
                if (x < nbc) dmp = prof[nbc - 1 - x];           /* columns overwrite rows */
                if (x >= Wp - nbc) dmp = prof[x - (Wp - nbc)];
                const size_t i = ((size_t)b * Hp + z) * Wp + x;
                const float vv = v[(size_t)z * Wp + x];
                float al = vv * dt; al = al / dx; al = al * al;
                const float kp = dmp * dt;
                float t1 = C1X2 * al; t1 = t1 + 2.0f; t1 = t1 - kp;
                float bt = vv * dt; bt = bt * bt;
                alpha[i] = al; kappa[i] = kp; temp1[i] = t1; temp2[i] = 1.0f - kp; beta[i] = bt;
            }
    }
    free(prof);
}

static inline int wrap(int i, int n) { i %= n; return i < 0 ? i + n : i; }

/* One forward step for one (b, s) slice: out = T1*p1 - T2*p0 + A*(c2*S1 + c3*S2), pde.py:79. */
static void fwd_step_slice(int Hp, int Wp, const float *al, const float *t1, const float *t2,
                           const float *p0, const float *p1, float *out)
{
    #pragma omp parallel for schedule(static)
    for (int z = 0; z < Hp; ++z) {
        const float *rm1 = p1 + (size_t)wrap(z - 1, Hp) * Wp, *rp1 = p1 + (size_t)wrap(z + 1, Hp) * Wp;
        const float *rm2 = p1 + (size_t)wrap(z - 2, Hp) * Wp, *rp2 = p1 + (size_t)wrap(z + 2, Hp) * Wp;
        const float *r0 = p1 + (size_t)z * Wp;
        for (int x = 0; x < Wp; ++x) {
            const size_t i = (size_t)z * Wp + x;
            const int xm1 = wrap(x - 1, Wp), xp1 = wrap(x + 1, Wp), xm2 = wrap(x - 2, Wp), xp2 = wrap(x + 2, Wp);
            float s1 = rm1[x] + rp1[x]; s1 = s1 + r0[xm1]; s1 = s1 + r0[xp1];
            float s2 = rm2[x] + rp2[x]; s2 = s2 + r0[xm2]; s2 = s2 + r0[xp2];
            float lap = C2 * s1; const float l2 = C3 * s2; lap = lap + l2;
            float a1 = t1[i] * p1[i]; const float a2 = t2[i] * p0[i]; a1 = a1 - a2;
            const float a3 = al[i] * lap;
            out[i] = a1 + a3;
        }
    }
}

/* Forward time loop (pde.py:74-86).  hist (nullable) receives P_j in slot j+1. */
void oracle_forward(const oracle_geom *g, const float *alpha, const float *temp1,
                    const float *temp2, const float *beta, float *seis, float *hist)
{
    const int Hp = Hp_of(g), Wp = Wp_of(g), nrec = oracle_nrec(g);
    const size_t N = (size_t)Hp * Wp, S = (size_t)g->B * g->ns * N;
    float *ring = NULL;
    if (!hist) { ring = (float *)calloc(3 * S, sizeof(float)); }
    else memset(hist, 0, 2 * S * sizeof(float));
    for (int i = 0; i < g->nt; ++i) {
        float *p0 = hist ? hist + (size_t)i * S : ring + (size_t)((i + 1) % 3) * S;   /* P_{i-1} */
        float *p1 = hist ? hist + (size_t)(i + 1) * S : ring + (size_t)((i + 2) % 3) * S; /* P_i */
        float *pn = hist ? hist + (size_t)(i + 2) * S : ring + (size_t)(i % 3) * S;       /* P_{i+1} */
        const float w = (float)g->wavelet[i];
        for (int b = 0; b < g->B; ++b)
            for (int s = 0; s < g->ns; ++s) {
                const size_t off = ((size_t)b * g->ns + s) * N;
                fwd_step_slice(Hp, Wp, alpha + b * N, temp1 + b * N, temp2 + b * N, p0 + off, p1 + off, pn + off);
                const size_t si = (size_t)g->isz * Wp + g->isx[s];
                const float add = beta[b * N + si] * w;      /* pde.py:81 */
                pn[off + si] = pn[off + si] + add;
                if (i % g->st == 0)
                    for (int r = 0; r < g->ng; ++r)                 /* pde.py:82-83 */
                        seis[(((size_t)b * g->ns + s) * nrec + i / g->st) * g->ng + r] =
                            pn[off + (size_t)g->igz * Wp + g->igx[r]];
            }
    }
    free(ring);
}

/*
 * Discrete adjoint.  Walks k = nt..1:
 *   L_k = T1*L_{k+1} - T2*L_{k+2} + (c2*N1(A*L_{k+1}) + c3*N2(A*L_{k+1})) + R^T dseis[k-1]
 *   gA_s(x) += L_k(x) * (2c1*P_{k-1}(x) + c2*N1(P_{k-1}) + c3*N2(P_{k-1}))     [per shot s]
 *   gKs     += sum_x (K(x) * P_{k-1}(x)) * (L_{k+1}(x) - L_k(x))   [fp32 terms, fp64 sum]
 *   gbeta[s]+= L_k(src_s) * w[k-1]
 * then gA = sum_s gA_s (s ascending, fp32).  Order: k descending per shot, then shots; the HIP
 * kernels use the same order and agree bit-for-bit on gA and gbeta.
 */
void oracle_adjoint(const oracle_geom *g, const float *alpha, const float *temp1,
                    const float *temp2, const float *kappa, const float *hist, const float *dseis,
                    float *gA, double *gKs, float *gbeta)
{
    const int Hp = Hp_of(g), Wp = Wp_of(g), nrec = oracle_nrec(g), ns = g->ns;
    const size_t N = (size_t)Hp * Wp, S = (size_t)g->B * ns * N;
    float *lam = (float *)calloc(3 * S, sizeof(float));
    float *q = (float *)malloc(S * sizeof(float));
    float *gAs = (float *)calloc(S, sizeof(float));
    for (int b = 0; b < g->B; ++b) gKs[b] = 0.0;
    memset(gbeta, 0, (size_t)g->B * ns * sizeof(float));
    for (int k = g->nt; k >= 1; --k) {
        float *L1 = lam + (size_t)((k + 1) % 3) * S;   /* L_{k+1} */
        float *L2 = lam + (size_t)((k + 2) % 3) * S;   /* L_{k+2} */
        float *L0 = lam + (size_t)(k % 3) * S;         /* L_k (overwrites L_{k+3}) */
        const float *P = hist + (size_t)k * S;         /* slot k = P_{k-1} */
        const int rec = ((k - 1) % g->st) == 0;
        const int kr = (k - 1) / g->st;
        for (int b = 0; b < g->B; ++b)
            for (int s = 0; s < ns; ++s) {
                const size_t off = ((size_t)b * ns + s) * N;
                for (size_t i = 0; i < N; ++i) q[off + i] = alpha[b * N + i] * L1[off + i];
            }
        for (int b = 0; b < g->B; ++b) {
            double ksum = 0.0;
            #pragma omp parallel for schedule(static) reduction(+:ksum)
            for (int z = 0; z < Hp; ++z) {
                const int zm1 = wrap(z - 1, Hp), zp1 = wrap(z + 1, Hp), zm2 = wrap(z - 2, Hp), zp2 = wrap(z + 2, Hp);
                for (int x = 0; x < Wp; ++x) {
                    const size_t i = (size_t)z * Wp + x, ci = b * N + i;
                    const int xm1 = wrap(x - 1, Wp), xp1 = wrap(x + 1, Wp), xm2 = wrap(x - 2, Wp), xp2 = wrap(x + 2, Wp);
                    for (int s = 0; s < ns; ++s) {
                        const size_t off = ((size_t)b * ns + s) * N;
                        const float *qq = q + off, *pp = P + off;
#define AT(arr, zz, xx) arr[(size_t)(zz) * Wp + (xx)]
                        float n1 = AT(qq, zm1, x) + AT(qq, zp1, x); n1 = n1 + AT(qq, z, xm1); n1 = n1 + AT(qq, z, xp1);
                        float n2 = AT(qq, zm2, x) + AT(qq, zp2, x); n2 = n2 + AT(qq, z, xm2); n2 = n2 + AT(qq, z, xp2);
                        float nb = C2 * n1; const float nb2 = C3 * n2; nb = nb + nb2;
                        float l = temp1[ci] * L1[off + i]; const float l2 = temp2[ci] * L2[off + i];
                        l = l - l2; l = l + nb;
                        if (rec && z == g->igz) {   /* R^T dseis: the column's receivers summed first
                                                       (index backward = index_put(accumulate) into zeros) */
                            int any = 0;
                            float dsum = 0.0f;
                            for (int r = 0; r < g->ng; ++r)
                                if (g->igx[r] == x) {
                                    const float d = dseis[(((size_t)b * ns + s) * nrec + kr) * g->ng + r];
                                    dsum = any ? dsum + d : d;
                                    any = 1;
                                }
                            if (any) l = l + dsum;
                        }
                        L0[off + i] = l;
                        float s1 = AT(pp, zm1, x) + AT(pp, zp1, x); s1 = s1 + AT(pp, z, xm1); s1 = s1 + AT(pp, z, xp1);
                        float s2 = AT(pp, zm2, x) + AT(pp, zp2, x); s2 = s2 + AT(pp, z, xm2); s2 = s2 + AT(pp, z, xp2);
#undef AT
                        float lap = C2 * s1; const float lp2 = C3 * s2; lap = lap + lp2;
                        float d = C1X2 * pp[i]; d = d + lap;
                        const float c = l * d;
                        gAs[off + i] = gAs[off + i] + c;
                        float kk = kappa[ci] * pp[i]; const float dl = L1[off + i] - l; kk = kk * dl;
                        ksum += (double)kk;   /* fp32 product (as autograd), fp64 sum */
                    }
                }
            }
            gKs[b] += ksum;
        }
        const float w = (float)g->wavelet[k - 1];
        for (int b = 0; b < g->B; ++b)
            for (int s = 0; s < ns; ++s) {
                const size_t off = ((size_t)b * ns + s) * N, si = (size_t)g->isz * Wp + g->isx[s];
                gbeta[b * ns + s] = gbeta[b * ns + s] + L0[off + si] * w;
            }
    }
    for (int b = 0; b < g->B; ++b)
        for (size_t i = 0; i < N; ++i) {
            float a = 0.0f;
            for (int s = 0; s < ns; ++s) a = a + gAs[((size_t)b * ns + s) * N + i];
            gA[b * N + i] = a;
        }
    free(lam); free(q); free(gAs);
}

/*
 * Velocity gradient from the adjoint accumulators (chain of pde.py:63-71, 38-52, 91 and
 * data_trans.py:13-15):
 *   g_vpad = gA * d(alpha)/dv + [src] gbeta * d(beta)/dv ;  g_vpad[argmin] += gKs / vmin
 *   g_v    = replicate-pad fold of g_vpad ;  g_vnorm = 1500 * g_v
 */
void oracle_grad_finalize(const oracle_geom *g, const float *vpad, const float *gA,
                          const double *gKs, const float *gbeta, const float *vmin,
                          const int64_t *argmin, float *gvnorm)
{
    const int Hp = Hp_of(g), Wp = Wp_of(g), nbc = g->nbc, nz = g->nz, nx = g->nx;
    const size_t N = (size_t)Hp * Wp;
    const float dt = g->dt, dx = g->dx;
    double *gv = (double *)malloc(N * sizeof(double));
    for (int b = 0; b < g->B; ++b) {
        const float *v = vpad + b * N;
        for (size_t i = 0; i < N; ++i) {
            float a1 = v[i] * dt; a1 = a1 / dx;
            float t = gA[b * N + i] * (2.0f * a1); t = t / dx; t = t * dt;
            gv[i] = t;
        }
        for (int s = 0; s < g->ns; ++s) {
            const size_t si = (size_t)g->isz * Wp + g->isx[s];
            const float b1 = v[si] * dt;
            float t = gbeta[b * g->ns + s] * (2.0f * b1); t = t * dt;
            gv[si] += t;
        }
        gv[argmin[b]] += gKs[b] / (double)vmin[b];
        for (int iz = 0; iz < nz; ++iz)
            for (int ix = 0; ix < nx; ++ix) {
                const int z0 = iz == 0 ? 0 : iz + nbc, z1 = iz == nz - 1 ? Hp : iz + nbc + 1;
                const int x0 = ix == 0 ? 0 : ix + nbc, x1 = ix == nx - 1 ? Wp : ix + nbc + 1;
                double acc = 0.0;   /* two-stage order: columns of a row, then rows */
                for (int z = z0; z < z1; ++z) {
                    double row = 0.0;
                    for (int x = x0; x < x1; ++x) row += gv[(size_t)z * Wp + x];
                    acc += row;
                }
                gvnorm[((size_t)b * nz + iz) * nx + ix] = (float)(acc * 1500.0);
            }
    }
    free(gv);
}
