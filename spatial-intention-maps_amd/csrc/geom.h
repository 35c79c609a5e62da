// geom.h -- exact fp64 geometry of the observation path, shared by host and device code.
//
// Everything here must round exactly like the reference's Python / numpy / scipy code, so the
// whole library is compiled with -ffp-contract=off; the single fused multiply-add is explicit
// (rotate out_center, see rot_params).  Citations are relative to the reference repo root.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#define SIMAPS_HD __host__ __device__ __forceinline__

namespace simaps {

constexpr int LW = 96;           // Mapper.LOCAL_MAP_PIXEL_WIDTH (envs.py:2011)
constexpr int CROP = 136;        // round_up_to_even(sqrt(2) * 96) (envs.py:2202)
constexpr int HALF_CROP = CROP / 2;
constexpr int TILE = CROP + 2;   // intention raster tile: crop + 1-px dilation halo
constexpr int TILE_HALF = TILE / 2;
constexpr double PPM = 96.0;     // Mapper.LOCAL_MAP_PIXELS_PER_METER
constexpr double RAD_TO_DEG = 180.0 / 3.141592653589793;  // CPython math.degrees: x * (180 / pi)

// Per-class robot geometry (envs.py:802-810, 1059-1062, 1279-1282), computed on the host with
// the reference's own expressions (see make_geometry in simaps.hip).
struct Geometry {
    double base_length[4];
    int cspace_r[4];    // floor(RADIUS * 96)                  (envs.py:2421)
    int mask_width[4];  // ceil(2 * RADIUS * 96)               (envs.py:2220)
    int mask_start[4];  // floor(96 / 2 - width / 2)           (envs.py:2222)
    int cube_w;         // ceil(CUBE_WIDTH * 96)               (envs.py:2225)
    int pad;
    double half_width, half_width_sq, backpack_offset;
    double cube_half, cube_width, cube_base;  // CUBE_WIDTH/2, CUBE_WIDTH, EE + LIFTED_CUBE_OFFSET
    // The 5 robot masks (types 0..3, 4 = lifting with lifted cube) as bit windows, filled on the
    // host from mask_bit(): mbits[m][r] bit c = mask[mrow0[m] + r][mcol0[m] + c].
    int mrow0[5], mcol0[5], mnrows[5], mncols[5];
    uint32_t mbits[5][24];
};

// ---- scipy.special.cosdg / sindg (cephes sindg.c) -----------------------------------------
SIMAPS_HD double polevl_(double x, const double *coef, int N)
{
    double ans = *coef++;
    int i = N;
    do { ans = ans * x + *coef++; } while (--i);
    return ans;
}

SIMAPS_HD double dg_core(double x, bool want_cos)
{
    const double sincof[] = {1.58962301572218447952E-10, -2.50507477628503540135E-8,
                             2.75573136213856773549E-6, -1.98412698295895384658E-4,
                             8.33333333332211858862E-3, -1.66666666666666307295E-1};
    const double coscof[] = {1.13678171382044553091E-11, -2.08758833757683644217E-9,
                             2.75573155429816611547E-7, -2.48015872936186303776E-5,
                             1.38888888888806666760E-3, -4.16666666666666348141E-2,
                             4.99999999999999999798E-1};
    const double PI180 = 1.74532925199432957692E-2;
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
    bool cos_poly = want_cos ? !((j == 1) || (j == 2)) : ((j == 1) || (j == 2));
    if (cos_poly) y = 1.0 - zz * polevl_(zz, coscof, 6);
    else y = z + z * (zz * polevl_(zz, sincof, 5));
    return sign < 0 ? -y : y;
}

// ---- scipy.ndimage.rotate(input n x n, angle, order=0, reshape=True) geometry ------------------
// scipy interpolation.py (1.7.1) 909-930; output pixel o samples input[floor(src + 0.5)] iff
// 0 <= src <= n-1 on both axes (else cval 0), src_r = (o0 * M[r][0] + o1 * M[r][1]) + off_r.
// out_center = M @ ((S-1)/2) goes through numpy matmul -> BLAS dgemv, whose rounding depends on the
// host's numpy / OpenBLAS build: fma(M[r][0], a0, M[r][1] * a1) (plain = false; pinned by
// tests/golden/rotate.npz) or M[r][0] * a0 + M[r][1] * a1 (plain = true; tests/golden/rotate_plain.npz).
struct Rot {
    double c, s, f0, f1;
    int S0, S1;
};

SIMAPS_HD Rot rot_params(int n, double angle, bool plain)
{
    Rot R;
    const double c = dg_core(angle, true), s = dg_core(angle, false);
    const double iy = n, ix = n;
    const double r0[4] = {0.0, s * ix, c * iy, c * iy + s * ix};
    const double r1[4] = {0.0, c * ix, -s * iy, -s * iy + c * ix};
    double mx0 = r0[0], mn0 = r0[0], mx1 = r1[0], mn1 = r1[0];
    for (int k = 1; k < 4; k++) {
        mx0 = r0[k] > mx0 ? r0[k] : mx0;
        mn0 = r0[k] < mn0 ? r0[k] : mn0;
        mx1 = r1[k] > mx1 ? r1[k] : mx1;
        mn1 = r1[k] < mn1 ? r1[k] : mn1;
    }
    R.S0 = (int)(mx0 - mn0 + 0.5);
    R.S1 = (int)(mx1 - mn1 + 0.5);
    const double a0 = (double)(R.S0 - 1) / 2, a1 = (double)(R.S1 - 1) / 2;
    const double oc0 = plain ? c * a0 + s * a1 : fma(c, a0, s * a1);
    const double oc1 = plain ? -s * a0 + c * a1 : fma(-s, a0, c * a1);
    const double inc = (double)(n - 1) / 2;
    R.c = c;
    R.s = s;
    R.f0 = inc - oc0;
    R.f1 = inc - oc1;
    return R;
}

// Source index of output pixel (o0, o1); false = outside (cval).
SIMAPS_HD bool rot_src(const Rot &R, int n, int o0, int o1, int &k0, int &k1)
{
    const double d0 = o0, d1 = o1;
    const double s0 = (d0 * R.c + d1 * R.s) + R.f0;
    const double s1 = (d0 * (-R.s) + d1 * R.c) + R.f1;
    const double hi = n - 1;
    if (!(s0 >= 0.0 && s0 <= hi && s1 >= 0.0 && s1 <= hi)) return false;
    k0 = (int)floor(s0 + 0.5);
    k1 = (int)floor(s1 + 0.5);
    return true;
}

// ---- Mapper.position_to_pixel_indices (envs.py:2391-2397) ----------------------------------------
SIMAPS_HD void pos_to_pix(double x, double y, int H, int W, int &pi, int &pj)
{
    double fi = floor((double)H / 2 - y * PPM);
    double fj = floor((double)W / 2 + x * PPM);
    int i = (int)fi, j = (int)fj;
    pi = i < 0 ? 0 : (i > H - 1 ? H - 1 : i);
    pj = j < 0 ? 0 : (j > W - 1 ? W - 1 : j);
}

// ---- Mapper._create_robot_mask (envs.py:2218-2242), one pixel --------------------------------------
SIMAPS_HD bool mask_bit(const Geometry &g, int type, bool with_cube, int i, int j)
{
    const int st = g.mask_start[type], wd = g.mask_width[type];
    const int i_lo = with_cube ? st - g.cube_w : st;
    if (i < i_lo || i >= st + wd || j < st || j >= st + wd) return false;
    const double px = ((j + 0.5) - (double)LW / 2) / PPM;  // pixel_indices_to_position (envs.py:2399-2403)
    const double py = ((double)LW / 2 - (i + 0.5)) / PPM;
    const double dy = py - g.backpack_offset;
    const bool in_base = fabs(px) <= g.half_width && 0 <= dy && dy <= g.base_length[type];
    const bool in_backpack = px * px + dy * dy <= g.half_width_sq;
    if (in_base || in_backpack) return true;
    if (with_cube) {
        const double cy = py - g.cube_base;
        return fabs(px) <= g.cube_half && 0 <= cy && cy <= g.cube_width;
    }
    return false;
}

}  // namespace simaps
