// tri_filter.h — the traversal's triangle record and its barycentric edge filter (host side).
//
// The reference decides "P inside the triangle" with three fp32 edge functions (RT:273-281):
//   e1 = dot(cross(p2 - p1, P - p1), N), e2 = ... (p3 - p2, P - p2), e3 = ... (p1 - p3, P - p3),
// hit iff all three > 0 or all three < 0.  That is ~60 VALU per test on the device.  The trace
// kernels instead evaluate two barycentric rows, b2 = R2.(P - p1), b3 = R3.(P - p1), b1 = 1 - b2 - b3
// (~20 VALU), and fall back to the reference's own three edge functions only when the filter cannot
// tell the sign of every e_k for certain.  Decisions therefore stay the reference's bit for bit.
//
// Why the signs agree (P = the computed hit point, D = max|P - p1|, u = 2^-24):
//   * With E2 = p2 - p1, E3 = p3 - p1, n = E2 x E3, P - p1 = b2 E2 + b3 E3 + h n^ (b's exact),
//     e1 = b3 (n.N) + h (E2 x n^).N, e2 = b1 (n.N) + ..., e3 = b2 (n.N) + ..., and n.N = |n| cos(th)
//     (th = angle between the fp32 N and the exact normal).  So sign(e_k) = sign(b_k) once |b_k|
//     exceeds the fp32 error of e_k, |h| |A| sin(th) / (|n| cos(th)) (|h| <= sqrt3 D) and
//     7u sum_i |N_i|(|A_j B_l| + |A_l B_j|) <= 24.3 u |A|inf |B|inf, |B|inf <= D + |A|inf (A: the
//     edge, B: P minus its start), all divided by |n| cos(th).
//   * b2~ = fl(R2f.(fl(P - p1))) is within 5u |R2|_1 D of b2 (rounding of R2, of P - p1 and the
//     three fma), b1~ within the sum of both plus 2u (1 + |b~|).
//   * |A|inf <= |n| (|R2|_1 + |R3|_1) and |R|_1 <= 3 max|R_i|, so with Lr = max|R2_i| + max|R3_i|
//     everything is bounded by  m = k1 * D * Lr + k0,
//       k1 = 2 (72.9 u / cos + 5.2 sin/cos + 50 u),  k0 = 2 (24.3 u S + 2 u),  S = |A|inf^2 / (|n| cos)
//     (maxima over the scene's triangles; factor 2 for the neglected higher-order terms).
//   * If min(b~) > m, every e_k has the sign of n.N: a hit.  If min(b~) < -m, that e_k has the other
//     sign while some b_j >= 1/2 > m (the b's sum to 1) keeps its sign: no hit.  Otherwise (or if
//     m >= 1/4) the kernel runs the reference's edge functions.
// Triangles whose S or sin/cos lie above the scene's 99.9th percentile or 16x its median (slivers)
// get zero rows:
// their b~ = (1, 0, 0) is never decisive, so they always take the reference's test, and the scene
// constants stay those of well-shaped triangles.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

namespace trif {

struct Consts {
  double k1 = 0.0, k0 = 0.0;
  int flagged = 0;  // triangles left to the reference's test alone
};

// tri: 3 float[4] per triangle {p1, N.x} {p2, N.y} {p3, N.z} (N = the reference's fp32 normal).
// out: 3 float[4] per triangle {p1, N.x} {R2, N.y} {R3, N.z}.
inline Consts build(const float* tri, long nt, float* out) {
  const double u = 0x1p-24;
  std::vector<double> S(nt, INFINITY), sc(nt, INFINITY), cs(nt, 0.0);
  for (long i = 0; i < nt; i++) {
    const float* A = tri + 12 * i;
    float* O = out + 12 * i;
    std::memcpy(O, A, 16);
    O[7] = A[7];
    O[11] = A[11];
    O[4] = O[5] = O[6] = O[8] = O[9] = O[10] = 0.0f;
    const double p1[3] = {A[0], A[1], A[2]}, p2[3] = {A[4], A[5], A[6]}, p3[3] = {A[8], A[9], A[10]};
    const double N[3] = {A[3], A[7], A[11]};
    if (!(std::isfinite(N[0]) && std::isfinite(N[1]) && std::isfinite(N[2]))) continue;  // never reaches the edges
    double E2[3], E3[3], E23[3];
    for (int a = 0; a < 3; a++) { E2[a] = p2[a] - p1[a]; E3[a] = p3[a] - p1[a]; E23[a] = p3[a] - p2[a]; }
    const double n[3] = {E2[1] * E3[2] - E2[2] * E3[1], E2[2] * E3[0] - E2[0] * E3[2], E2[0] * E3[1] - E2[1] * E3[0]};
    const double nn2 = n[0] * n[0] + n[1] * n[1] + n[2] * n[2], nn = std::sqrt(nn2);
    if (!(nn > 0.0) || !std::isfinite(nn2)) continue;
    const double c = (N[0] * n[0] + N[1] * n[1] + N[2] * n[2]) / nn;
    const double x[3] = {N[1] * n[2] - N[2] * n[1], N[2] * n[0] - N[0] * n[2], N[0] * n[1] - N[1] * n[0]};
    const double s = std::sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]) / nn;
    if (!(c > 0.5)) continue;
    double amax = 0.0;
    for (int a = 0; a < 3; a++) amax = std::max({amax, std::fabs(E2[a]), std::fabs(E3[a]), std::fabs(E23[a])});
    const double R2[3] = {(E3[1] * n[2] - E3[2] * n[1]) / nn2, (E3[2] * n[0] - E3[0] * n[2]) / nn2,
                          (E3[0] * n[1] - E3[1] * n[0]) / nn2};
    const double R3[3] = {(n[1] * E2[2] - n[2] * E2[1]) / nn2, (n[2] * E2[0] - n[0] * E2[2]) / nn2,
                          (n[0] * E2[1] - n[1] * E2[0]) / nn2};
    bool fin = true;
    for (int a = 0; a < 3; a++) fin = fin && std::isfinite((float)R2[a]) && std::isfinite((float)R3[a]);
    if (!fin) continue;
    for (int a = 0; a < 3; a++) { O[4 + a] = (float)R2[a]; O[8 + a] = (float)R3[a]; }
    S[i] = amax * amax / (nn * c);
    sc[i] = s / c;
    cs[i] = c;
  }
  // cap: the 99.9th percentile, but at most 16x the median (a scene with many slivers keeps the
  // margin of its well-shaped triangles; the slivers take the reference's test)
  auto cap = [&](const std::vector<double>& v, double floor_) {
    std::vector<double> f;
    for (double x : v) if (std::isfinite(x)) f.push_back(x);
    if (f.empty()) return floor_;
    const size_t k = std::min(f.size() - 1, (size_t)(0.999 * (double)f.size()));
    std::nth_element(f.begin(), f.begin() + (long)k, f.end());
    const double hi = f[k];
    std::nth_element(f.begin(), f.begin() + (long)(f.size() / 2), f.end());
    return std::max(floor_, std::min(hi, 16.0 * f[f.size() / 2]));
  };
  const double s_cap = cap(S, 8.0), sc_cap = cap(sc, 4.0 * u);
  Consts k;
  double s_max = 0.0, sc_max = 0.0, c_min = 1.0;
  for (long i = 0; i < nt; i++) {
    float* O = out + 12 * i;
    if (!(S[i] <= s_cap && sc[i] <= sc_cap)) {
      O[4] = O[5] = O[6] = O[8] = O[9] = O[10] = 0.0f;
      k.flagged++;
      continue;
    }
    s_max = std::max(s_max, S[i]);
    sc_max = std::max(sc_max, sc[i]);
    c_min = std::min(c_min, cs[i]);
  }
  k.k1 = 2.0 * (72.9 * u / c_min + 5.2 * sc_max + 50.0 * u);
  k.k0 = 2.0 * (24.3 * u * s_max + 2.0 * u);
  return k;
}

}  // namespace trif
