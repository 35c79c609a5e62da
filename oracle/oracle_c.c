/* oracle_c.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * Plain-C restatements of the integer / float kernels of the observation path that live in
 * native code in the reference or its dependencies.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg load this library (through oracle/oracle.py).
 *
 * Pinned against tests/golden/{sssp,edt,trig}.npz, which were produced by the reference itself
 * (tests/golden/make_goldens.py).  Build: `make -C oracle` (gcc -ffp-contract=off).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------
 * GridGraph + SPFA  (shortest_paths/shortest_paths.pyx:24-67 graph build, 69-114 _spfa)
 * 8-neighbour graph over cells with grid != 0, direction order and weights as pyx:30-32,
 * float32 relaxation with strict '<', SLF swap (pyx:104-107), unreachable -> -1 (pyx:110-112).
 * Returns 0, or -1 if the queue would overflow (the reference does not check; it sizes the
 * queue V*8 as we do).
 * ------------------------------------------------------------------------------------------ */
int oracle_spfa(const uint8_t *grid, int H, int W, int si, int sj, float *dists, int32_t *parents)
{
    static const int dirs[8][2] = {{0, -1}, {0, 1}, {-1, -1}, {-1, 0}, {-1, 1}, {1, -1}, {1, 0}, {1, 1}};
    const float sqrt_2 = (float)1.4142135623730951; /* np.sqrt(2) stored into a C float */
    const float dir_lengths[8] = {1, 1, sqrt_2, 1, sqrt_2, sqrt_2, 1, sqrt_2};
    const int V = H * W;
    const float inf = (float)(2 * V);
    int32_t *edges = (int32_t *)malloc(sizeof(int32_t) * (size_t)V * 8);
    float *weights = (float *)malloc(sizeof(float) * (size_t)V * 8);
    int32_t *counts = (int32_t *)calloc((size_t)V, sizeof(int32_t));
    int32_t *queue = (int32_t *)malloc(sizeof(int32_t) * ((size_t)V * 8 + 1));
    int32_t *in_queue = (int32_t *)calloc((size_t)V, sizeof(int32_t));
    int rc = 0;
    for (int i = 0; i < H; i++)
        for (int j = 0; j < W; j++) {
            int v = i * W + j;
            if (grid[v] == 0) continue;
            for (int k = 0; k < 8; k++) {
                int ip = i + dirs[k][0], jp = j + dirs[k][1];
                if (ip < 0 || jp < 0 || ip >= H || jp >= W || grid[ip * W + jp] == 0) continue;
                int e = v * 8 + counts[v];
                edges[e] = ip * W + jp;
                weights[e] = dir_lengths[k];
                counts[v] += 1;
            }
        }
    for (int v = 0; v < V; v++) { dists[v] = inf; parents[v] = -1; }
    long head = 0, tail = 0, cap = (long)V * 8;
    int s = si * W + sj;
    dists[s] = 0;
    tail += 1;
    queue[tail] = s;
    in_queue[s] = 1;
    while (head < tail) {
        head += 1;
        int u = queue[head];
        in_queue[u] = 0;
        for (int k = 0; k < counts[u]; k++) {
            int e = u * 8 + k;
            int v = edges[e];
            float new_dist = dists[u] + weights[e];
            if (new_dist < dists[v]) {
                parents[v] = u;
                dists[v] = new_dist;
                if (!in_queue[v]) {
                    if (tail + 1 >= cap) { rc = -1; goto done; }
                    tail += 1;
                    queue[tail] = v;
                    in_queue[v] = 1;
                    if (dists[queue[tail]] < dists[queue[head + 1]]) {
                        int tmp = queue[tail];
                        queue[tail] = queue[head + 1];
                        queue[head + 1] = tmp;
                    }
                }
            }
        }
    }
    for (int v = 0; v < V; v++)
        if ((double)dists[v] >= (double)inf - 1e-6) dists[v] = -1;
done:
    free(edges); free(weights); free(counts); free(queue); free(in_queue);
    return rc;
}

/* ------------------------------------------------------------------------------------------
 * scipy.ndimage.distance_transform_edt(..., return_indices=True) feature transform, rank 2.
 * Restates scipy's ni_morphology.c (_ComputeFT / _VoronoiFT, Maurer-style separable Voronoi
 * FT): pass 1 per column along axis 0, pass 2 per row along axis 1.  Feature points are the
 * ZERO pixels of `img`.  All arithmetic is on small integers, so int64 is exact.
 * ft[0*H*W + p] = row, ft[1*H*W + p] = col.  Pixels with no feature anywhere keep -1 / 0.
 * ------------------------------------------------------------------------------------------ */
static void voronoi_ft_row(int32_t *f0, int32_t *f1, int len, int d, int64_t coor_other, int32_t *g)
{
    /* f0/f1: per-position component 0/1 (in place).  d = axis processed (0 or 1). */
    long l = -1;
    int32_t *fd_arr = d == 0 ? f0 : f1;   /* component along d   */
    int32_t *fo_arr = d == 0 ? f1 : f0;   /* the other component */
    for (int ii = 0; ii < len; ii++) {
        if (f0[ii] < 0) continue;
        int64_t fd = fd_arr[ii];
        int64_t tw = (int64_t)fo_arr[ii] - coor_other;
        int64_t wR = tw * tw;
        while (l >= 1) {
            int idx1 = g[l], idx2 = g[l - 1];
            int64_t f1d = fd_arr[idx1];
            int64_t a = f1d - fd_arr[idx2];
            int64_t b = fd - f1d;
            int64_t tu = (int64_t)fo_arr[idx2] - coor_other, tv = (int64_t)fo_arr[idx1] - coor_other;
            int64_t uR = tu * tu, vR = tv * tv;
            int64_t c = a + b;
            if (c * vR - b * uR - a * wR - a * b * c <= 0) break;
            --l;
        }
        ++l;
        g[l] = ii;
    }
    long maxl = l;
    if (maxl < 0) return;
    /* copy the envelope's features before overwriting */
    int32_t *c0 = (int32_t *)malloc(sizeof(int32_t) * (size_t)(maxl + 1));
    int32_t *c1 = (int32_t *)malloc(sizeof(int32_t) * (size_t)(maxl + 1));
    for (long q = 0; q <= maxl; q++) { c0[q] = f0[g[q]]; c1[q] = f1[g[q]]; }
    l = 0;
    for (int ii = 0; ii < len; ii++) {
        int64_t t0, t1;
        t0 = d == 0 ? (int64_t)c0[l] - ii : (int64_t)c0[l] - coor_other;
        t1 = d == 1 ? (int64_t)c1[l] - ii : (int64_t)c1[l] - coor_other;
        int64_t delta1 = t0 * t0 + t1 * t1;
        while (l < maxl) {
            t0 = d == 0 ? (int64_t)c0[l + 1] - ii : (int64_t)c0[l + 1] - coor_other;
            t1 = d == 1 ? (int64_t)c1[l + 1] - ii : (int64_t)c1[l + 1] - coor_other;
            int64_t delta2 = t0 * t0 + t1 * t1;
            if (delta1 <= delta2) break;
            delta1 = delta2;
            ++l;
        }
        f0[ii] = c0[l];
        f1[ii] = c1[l];
    }
    free(c0); free(c1);
}

void oracle_edt_ft(const uint8_t *img, int H, int W, int32_t *ft)
{
    int32_t *F0 = ft, *F1 = ft + (size_t)H * W;
    int n = H > W ? H : W;
    int32_t *a0 = (int32_t *)malloc(sizeof(int32_t) * n), *a1 = (int32_t *)malloc(sizeof(int32_t) * n);
    int32_t *g = (int32_t *)malloc(sizeof(int32_t) * n);
    memset(F1, 0, sizeof(int32_t) * (size_t)H * W);
    /* pass 1: each column j, along axis 0 */
    for (int j = 0; j < W; j++) {
        for (int i = 0; i < H; i++) {
            if (img[i * W + j]) { a0[i] = -1; a1[i] = 0; }
            else { a0[i] = i; a1[i] = j; }
        }
        voronoi_ft_row(a0, a1, H, 0, j, g);
        for (int i = 0; i < H; i++) { F0[i * W + j] = a0[i]; F1[i * W + j] = a1[i]; }
    }
    /* pass 2: each row i, along axis 1 */
    for (int i = 0; i < H; i++) {
        for (int j = 0; j < W; j++) { a0[j] = F0[i * W + j]; a1[j] = F1[i * W + j]; }
        voronoi_ft_row(a0, a1, W, 1, i, g);
        for (int j = 0; j < W; j++) { F0[i * W + j] = a0[j]; F1[i * W + j] = a1[j]; }
    }
    free(a0); free(a1); free(g);
}

/* ------------------------------------------------------------------------------------------
 * scipy.special.cosdg / sindg (cephes sindg.c; scipy/special/xsf/cephes/sindg.h), used by
 * scipy.ndimage.rotate.  Compiled with -ffp-contract=off: no FMA, exactly the cephes ops.
 * ------------------------------------------------------------------------------------------ */
static const double sincof[] = {1.58962301572218447952E-10, -2.50507477628503540135E-8,
                                2.75573136213856773549E-6, -1.98412698295895384658E-4,
                                8.33333333332211858862E-3, -1.66666666666666307295E-1};
static const double coscof[] = {1.13678171382044553091E-11, -2.08758833757683644217E-9,
                                2.75573155429816611547E-7, -2.48015872936186303776E-5,
                                1.38888888888806666760E-3, -4.16666666666666348141E-2,
                                4.99999999999999999798E-1};
static const double PI180 = 1.74532925199432957692E-2;

static double polevl(double x, const double *coef, int N)
{
    double ans = *coef++;
    int i = N;
    do { ans = ans * x + *coef++; } while (--i);
    return ans;
}

static double dg_core(double x, int want_cos)
{
    double y, z, zz;
    int j, sign = 1;
    if (x < 0) { x = -x; if (!want_cos) sign = -1; }
    if (x > 1.0e14) return 0.0;
    y = floor(x / 45.0);
    z = ldexp(y, -4);
    z = floor(z);
    z = y - ldexp(z, 4);
    j = (int)z;
    if (j & 1) { j += 1; y += 1.0; }
    j = j & 07;
    if (j > 3) { sign = -sign; j -= 4; }
    if (want_cos && j > 1) sign = -sign;
    z = x - y * 45.0;
    z *= PI180;
    zz = z * z;
    int use_cos_poly = want_cos ? !((j == 1) || (j == 2)) : ((j == 1) || (j == 2));
    if (use_cos_poly) y = 1.0 - zz * polevl(zz, coscof, 6);
    else y = z + z * (zz * polevl(zz, sincof, 5));
    if (sign < 0) y = -y;
    return y;
}

double oracle_sindg(double x) { return dg_core(x, 0); }
double oracle_cosdg(double x) { return dg_core(x, 1); }

/* ------------------------------------------------------------------------------------------
 * scipy.ndimage.rotate(reshape=True) geometry for an n x n input (scipy interpolation.py:909-930)
 *   out_bounds = M @ [[0,0,n,n],[0,n,0,n]] -> S = int(ptp + 0.5)        (plain products/sums)
 *   out_center = M @ ((S - 1) / 2)                                        (numpy matmul -> BLAS
 *       dgemv, whose rounding is a property of the host's numpy / OpenBLAS build:
 *       plain == 0: fma(M[r][0], a0, M[r][1] * a1) -- the FMA kernel (numpy 2.2.6 here; the
 *                   round-1 builder host's numpy 1.26.4), pinned by tests/golden/rotate.npz;
 *       plain == 1: M[r][0] * a0 + M[r][1] * a1 -- numpy 1.26.4 / OpenBLAS 0.3.23 on this
 *                   AVX-512 Xeon, pinned by tests/golden/rotate_plain.npz.
 *       Each form matches its host on every golden angle and the other on only ~50-55 % of
 *       them, ~4 % of random headings giving a different sample grid.)
 *   offset = (n - 1) / 2 - out_center
 * out: {S0, S1, c, s, off0, off1}
 * ------------------------------------------------------------------------------------------ */
void oracle_rotate_params(int n, double angle, int plain, double *out)
{
    double c = oracle_cosdg(angle), s = oracle_sindg(angle);
    double iy = n, ix = n;
    double r0[4] = {0.0, s * ix, c * iy, c * iy + s * ix};
    double r1[4] = {0.0, c * ix, -s * iy, -s * iy + c * ix};
    double mx0 = r0[0], mn0 = r0[0], mx1 = r1[0], mn1 = r1[0];
    for (int k = 1; k < 4; k++) {
        if (r0[k] > mx0) mx0 = r0[k];
        if (r0[k] < mn0) mn0 = r0[k];
        if (r1[k] > mx1) mx1 = r1[k];
        if (r1[k] < mn1) mn1 = r1[k];
    }
    long S0 = (long)(mx0 - mn0 + 0.5), S1 = (long)(mx1 - mn1 + 0.5);
    double a0 = (double)(S0 - 1) / 2, a1 = (double)(S1 - 1) / 2;
    double oc0 = plain ? c * a0 + s * a1 : fma(c, a0, s * a1);
    double oc1 = plain ? -s * a0 + c * a1 : fma(-s, a0, c * a1);
    double inc = (double)(n - 1) / 2;
    out[0] = (double)S0; out[1] = (double)S1; out[2] = c; out[3] = s;
    out[4] = inc - oc0; out[5] = inc - oc1;
}
