// rt_device.h — device-side building blocks of the MI355X path tracer (HIP, gfx950).
//
// Scalar fp32 restatement of the shading math of the reference fragment shader
// (src/shaders/fragment_shader_ray_tracing.glsl, "RT:<line>").  Evaluation order is kept
// operator-for-operator (no FMA contraction: built with -ffp-contract=off) and every GLSL
// builtin goes through glsl_math.h, so the kernel reproduces the CPU oracle bit for bit.
// Data access is MI355X-shaped instead of texel-shaped: 16-B float4 loads from SoA-ish
// arrays (see DESIGN.md "Data layout in HBM").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "glsl_math.h"

#pragma clang fp contract(off)

#define RTD __device__ __forceinline__

namespace rtd {
using namespace gm;

// ------------------------------------------------------------------------- f3 vector
struct f3 {
  float x, y, z;
};
RTD f3 mk3(float x, float y, float z) { return f3{x, y, z}; }
RTD f3 splat(float a) { return f3{a, a, a}; }
RTD f3 operator+(f3 a, f3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
RTD f3 operator-(f3 a, f3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
RTD f3 operator*(f3 a, f3 b) { return mk3(a.x * b.x, a.y * b.y, a.z * b.z); }
RTD f3 operator/(f3 a, f3 b) { return mk3(a.x / b.x, a.y / b.y, a.z / b.z); }
RTD f3 operator*(f3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
RTD f3 operator*(float s, f3 a) { return mk3(s * a.x, s * a.y, s * a.z); }
RTD f3 operator/(f3 a, float s) { return mk3(a.x / s, a.y / s, a.z / s); }
RTD f3 operator-(f3 a) { return mk3(-a.x, -a.y, -a.z); }
RTD float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
RTD f3 cross(f3 a, f3 b) { return mk3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y); }
RTD f3 normalize(f3 v) {
  float inv = 1.0f / sqrt_(dot(v, v));
  return v * inv;
}
RTD f3 mix(f3 x, f3 y, float a) { return x * (1.0f - a) + y * a; }
RTD f3 exp3(f3 v) { return mk3(exp_(v.x), exp_(v.y), exp_(v.z)); }
RTD f3 reflect(f3 I, f3 N) { return I - 2.0f * dot(N, I) * N; }
RTD f3 refract(f3 I, f3 N, float eta) {
  float k = 1.0f - eta * eta * (1.0f - dot(N, I) * dot(N, I));
  if (k < 0.0f) return splat(0.0f);
  return eta * I - (eta * dot(N, I) + sqrt_(k)) * N;
}
RTD f3 xyz(float4 v) { return mk3(v.x, v.y, v.z); }

constexpr float PI = 3.14159265358979323f;
constexpr float INV_PI = 0.31830988618379067f;
constexpr float TWO_PI = 6.28318530717958648f;
constexpr float INV_4_PI = 0.07957747154594766f;
constexpr float INF = 114514.0f;
constexpr int MEDIUM_ABSORB = 1, MEDIUM_SCATTER = 2, MEDIUM_EMISSIVE = 3;

// ------------------------------------------------------------------------ device data
// BVH node in "children-in-parent" form: the two child boxes the reference fetches with
// getBVHNode(node.left/right) (RT:363-370) live in the parent's 64-B record, and children
// are references (internal index, or a leaf's triangle range) so a leaf costs no fetch.
struct __attribute__((aligned(16))) GNode {
  float4 b0;  // L.AA.xyz, L.BB.x
  float4 b1;  // L.BB.yz,  R.AA.xy
  float4 b2;  // R.AA.z,   R.BB.xyz
  int4 ref;   // left ref, right ref, -, -
};
// 4-wide node collapsed from the binary tree above (same exact fp32 child boxes, SoA: child k
// in component k; an empty slot has the inverted bounds lo = +inf, hi = -inf and the ref Q_EMPTY).
// The sign-selected slab of a ray with a finite 1/d never hits an inverted box (t0 = +inf,
// t1 = -inf).  The literal slab of a ray with a zero direction component takes per-axis min / max,
// which turns the inverted box into an infinite one, so that path tests the slot's ref instead
// (tl_qnode_keys, coop_box): entering a Q_EMPTY ref reads QNode 0x7fffffff, far outside the
// array (the round-4 hipErrorIllegalAddress).  128 B = one cache line; one fetch
// replaces about two dependent binary steps.
struct __attribute__((aligned(16))) QNode {
  float4 lox, loy, loz, hix, hiy, hiz;
  int4 ref;  // child refs (QNode index or leaf ref), Q_EMPTY for an empty slot
  int4 pad;
};
static_assert(sizeof(QNode) == 128, "one cache line");
constexpr int Q_EMPTY = 0x7fffffff;
constexpr uint32_t LEAF_BIT = 0x80000000u;
RTD bool ref_is_leaf(int r) { return ((uint32_t)r & LEAF_BIT) != 0u; }
RTD int leaf_first(int r) { return (int)(((uint32_t)r & 0x7fffffffu) >> 4); }
RTD int leaf_count(int r) { return (int)((uint32_t)r & 15u) + 1; }

// Material table entry: 32 floats (the 24 Material.h floats, then ax, ay precomputed by
// getMaterial's formula RT:205-207, then the int medium type).
struct Mat {
  f3 emissive, baseColor;
  float subsurface, metallic, specular, specularTint, roughness, anisotropic, sheen, sheenTint, clearcoat,
      clearcoatGloss, IOR, transmission, ax, ay;
  int mtype;
  float mdensity, manis;
  f3 mcolor;
};
RTD Mat load_mat(const float4* __restrict__ mats, int id) {
  const float4* p = mats + 8 * id;
  float4 a = p[0], b = p[1], c = p[2], d = p[3], e = p[4], f = p[5], g = p[6];
  Mat m;
  m.emissive = mk3(a.x, a.y, a.z);
  m.baseColor = mk3(a.w, b.x, b.y);
  m.subsurface = b.z; m.metallic = b.w; m.specular = c.x; m.specularTint = c.y;
  m.roughness = c.z; m.anisotropic = c.w; m.sheen = d.x; m.sheenTint = d.y;
  m.clearcoat = d.z; m.clearcoatGloss = d.w; m.IOR = e.x; m.transmission = e.y;
  m.mcolor = mk3(e.z, e.w, f.x);
  m.mdensity = f.z; m.manis = f.w;
  m.ax = g.x; m.ay = g.y;
  m.mtype = __float_as_int(g.z);
  return m;
}

// ------------------------------------------------------------------ env textures (R13)
// texture() with NEAREST + CLAMP_TO_EDGE on W x H float4 texels.
RTD unsigned int tex_index(int w, int h, float u, float v) {
  int i = (int)floor_(u * (float)w);
  int j = (int)floor_(v * (float)h);
  if (isnan_(u)) i = 0;
  if (isnan_(v)) j = 0;
  i = i < 0 ? 0 : (i > w - 1 ? w - 1 : i);
  j = j < 0 ? 0 : (j > h - 1 ? h - 1 : j);
  return (unsigned int)j * (unsigned int)w + (unsigned int)i;
}
template <class T>
RTD T tex_nearest(const T* __restrict__ img, int w, int h, float u, float v) {
  return img[tex_index(w, h, u, v)];
}

// hdr texel = {hdrMap.rgb, hdrCache.b (pdf)}: hdrColor and hdrPdf of a direction read the same
// texel of both maps (RT:1165-1186), so one 16-B fetch serves both; cache = hdrCache.rg, the
// inverse-CDF sample of SampleHdr (RT:636).  Same values as the two RGB32F textures.
struct Env {
  const float4* __restrict__ hdr;
  const float2* __restrict__ cache;
  const float4* __restrict__ light;  // per cache texel: {L, hdrPdf(L)}, {hdrColor(L), 0} (rt_light_table_kernel)
  int w, h, res;
  float angle, intensity;
};

RTD void toSphericalCoord(const Env& E, f3 v, float& u, float& w) {  // RT:625-631
  float ux = atan2_(v.z, v.x), uy = asin_(v.y);
  ux = ux / (2.0f * PI);
  uy = uy / PI;
  ux = ux + 0.5f;
  uy = uy + 0.5f;
  uy = 1.0f - uy;
  u = ux + E.angle;
  w = uy + 0.0f;
}
RTD f3 SampleHdrTexel(float2 c) {  // RT:637-645: the direction of one hdrCache texel
  float x = c.x;
  float y = 1.0f - c.y;
  float phi = 2.0f * PI * (x - 0.5f);
  float theta = PI * (y - 0.5f);
  float st, ct, sp, cp;
  sincos_(theta, &st, &ct);
  sincos_(phi, &sp, &cp);
  return mk3(ct * cp, st, ct * sp);
}
RTD f3 SampleHdr(const Env& E, float xi_1, float xi_2) {  // RT:635-646
  return SampleHdrTexel(tex_nearest(E.cache, E.w, E.h, xi_1, xi_2));
}
RTD f3 hdrColor(const Env& E, f3 L) {  // RT:1165-1169
  float u, v;
  toSphericalCoord(E, normalize(L), u, v);
  return xyz(tex_nearest(E.hdr, E.w, E.h, u, v));
}
RTD float hdrPdf(const Env& E, f3 L) {  // RT:1173-1186
  float u, v;
  toSphericalCoord(E, normalize(L), u, v);
  float pdf = tex_nearest(E.hdr, E.w, E.h, u, v).w;
  float theta = PI * v;
  float sin_theta = max_(sin_(theta), 1e-10f);
  float p_convert = (float)(E.res * E.res / 2) / (TWO_PI * PI * sin_theta);
  return pdf * p_convert;
}
// hdrColor + hdrPdf of the same direction share one spherical mapping (same values).
RTD void hdrColorPdf(const Env& E, f3 L, f3& color, float& pdfv) {
  float u, v;
  toSphericalCoord(E, normalize(L), u, v);
  const float4 t = tex_nearest(E.hdr, E.w, E.h, u, v);
  color = xyz(t);
  float pdf = t.w;
  float theta = PI * v;
  float sin_theta = max_(sin_(theta), 1e-10f);
  float p_convert = (float)(E.res * E.res / 2) / (TWO_PI * PI * sin_theta);
  pdfv = pdf * p_convert;
}
// The NEE light sample of RT:1382-1392 from the per-texel table: SampleHdr(xi_1, xi_2) and
// hdrColor / hdrPdf of that direction depend only on the hdrCache texel the sample lands on, so
// rt_light_table_kernel evaluates them once per texel with the same functions (same bits) and a
// sample costs one 32-B fetch instead of a texel fetch, two sincos, atan2, asin, sin and a
// second, dependent texel fetch
RTD void SampleHdrLight(const Env& E, float xi_1, float xi_2, f3& L, f3& color, float& pdf) {
  const float4* t = E.light + 2u * (size_t)tex_index(E.w, E.h, xi_1, xi_2);
  const float4 a = t[0], b = t[1];
  L = xyz(a);
  pdf = a.w;
  color = xyz(b);
}
RTD f3 getDefaultSkyColor(float y) {  // RT:1190-1193
  float t = 0.5f * (y + 1.0f);
  return (1.0f - t) * mk3(1.0f, 1.0f, 1.0f) + t * mk3(0.5f, 0.7f, 1.0f);
}

// ------------------------------------------------------------------------------ RNG
RTD float rand_(uint32_t& wseed) {  // RT:577-586 (Thomas Wang hash)
  uint32_t seed = wseed;
  seed = (seed ^ 61u) ^ (seed >> 16u);
  seed *= 9u;
  seed = seed ^ (seed >> 4u);
  seed *= 0x27d4eb2du;
  wseed = seed ^ (seed >> 15u);
  return (float)wseed * (1.0f / 4294967296.0f);
}
__constant__ uint32_t kSobolV[8 * 32] = {
2147483648u, 1073741824u, 536870912u, 268435456u, 134217728u, 67108864u, 33554432u, 16777216u, 8388608u, 4194304u, 2097152u, 1048576u, 524288u, 262144u, 131072u, 65536u, 32768u, 16384u, 8192u, 4096u, 2048u, 1024u, 512u, 256u, 128u, 64u, 32u, 16u, 8u, 4u, 2u, 1u,
2147483648u, 3221225472u, 2684354560u, 4026531840u, 2281701376u, 3422552064u, 2852126720u, 4278190080u, 2155872256u, 3233808384u, 2694840320u, 4042260480u, 2290614272u, 3435921408u, 2863267840u, 4294901760u, 2147516416u, 3221274624u, 2684395520u, 4026593280u, 2281736192u, 3422604288u, 2852170240u, 4278255360u, 2155905152u, 3233857728u, 2694881440u, 4042322160u, 2290649224u, 3435973836u, 2863311530u, 4294967295u,
2147483648u, 3221225472u, 1610612736u, 2415919104u, 3892314112u, 1543503872u, 2382364672u, 3305111552u, 1753219072u, 2629828608u, 3999268864u, 1435500544u, 2154299392u, 3231449088u, 1626210304u, 2421489664u, 3900735488u, 1556135936u, 2388680704u, 3314585600u, 1751705600u, 2627492864u, 4008611328u, 1431684352u, 2147543168u, 3221249216u, 1610649184u, 2415969680u, 3892340840u, 1543543964u, 2382425838u, 3305133397u,
2147483648u, 3221225472u, 536870912u, 1342177280u, 4160749568u, 1946157056u, 2717908992u, 2466250752u, 3632267264u, 624951296u, 1507852288u, 3872391168u, 2013790208u, 3020685312u, 2181169152u, 3271884800u, 546275328u, 1363623936u, 4226424832u, 1977167872u, 2693105664u, 2437829632u, 3689389568u, 635137280u, 1484783744u, 3846176960u, 2044723232u, 3067084880u, 2148008184u, 3222012020u, 537002146u, 1342505107u,
2147483648u, 1073741824u, 536870912u, 2952790016u, 4160749568u, 3690987520u, 2046820352u, 2634022912u, 1518338048u, 801112064u, 2707423232u, 4038066176u, 3666345984u, 1875116032u, 2170683392u, 1085997056u, 579305472u, 3016343552u, 4217741312u, 3719483392u, 2013407232u, 2617981952u, 1510979072u, 755882752u, 2726789248u, 4090085440u, 3680870432u, 1840435376u, 2147625208u, 1074478300u, 537900666u, 2953698205u,
2147483648u, 1073741824u, 1610612736u, 805306368u, 2818572288u, 335544320u, 2113929216u, 3472883712u, 2290089984u, 3829399552u, 3059744768u, 1127219200u, 3089629184u, 4199809024u, 3567124480u, 1891565568u, 394297344u, 3988799488u, 920674304u, 4193267712u, 2950604800u, 3977188352u, 3250028032u, 129093376u, 2231568512u, 2963678272u, 4281226848u, 432124720u, 803643432u, 1633613396u, 2672665246u, 3170194367u,
2147483648u, 3221225472u, 2684354560u, 3489660928u, 1476395008u, 2483027968u, 1040187392u, 3808428032u, 3196059648u, 599785472u, 505413632u, 4077912064u, 1182269440u, 1736704000u, 2017853440u, 2221342720u, 3329785856u, 2810494976u, 3628507136u, 1416089600u, 2658719744u, 864310272u, 3863387648u, 3076993792u, 553150080u, 272922560u, 4167467040u, 1148698640u, 1719673080u, 2009075780u, 2149644390u, 3222291575u,
2147483648u, 1073741824u, 2684354560u, 1342177280u, 2281701376u, 1946157056u, 436207616u, 2566914048u, 2625634304u, 3208642560u, 2720006144u, 2098200576u, 111673344u, 2354315264u, 3464626176u, 4027383808u, 2886631424u, 3770826752u, 1691164672u, 3357462528u, 1993345024u, 3752330240u, 873073152u, 2870150400u, 1700563072u, 87021376u, 1097028000u, 1222351248u, 1560027592u, 2977959924u, 23268898u, 437609937u};

// sobol(d, grayCode(i)) RT:598-612; V reads at d >= 8 fall outside the table -> 0 (R8)
RTD float sobol_gray(int d, int g) {
  uint32_t result = 0u;
  if (d < 8) {
    int offset = d * 32;
    for (int j = 0; g != 0; g >>= 1, j++)
      if ((g & 1) != 0) result ^= kSobolV[j + offset];
  }
  return (float)result * (1.0f / 4294967296.0f);
}

// --------------------------------------------------------------------- Disney BSDF
RTD float sqr(float x) { return x * x; }
RTD float Luminance(f3 c) { return 0.212671f * c.x + 0.715160f * c.y + 0.072169f * c.z; }

RTD void getTangent(f3 N, f3& tangent, f3& bitangent) {  // RT:396-407
  f3 helper = mk3(1, 0, 0);
  if (fabs_(N.x) > 0.999f) helper = mk3(0, 0, 1);
  bitangent = normalize(cross(N, helper));
  tangent = normalize(cross(N, bitangent));
}
RTD void GetSpecColor(const Mat& mat, float eta, f3& specCol, f3& sheenCol) {  // RT:420-427
  float luminance = Luminance(mat.baseColor);
  f3 ctint = luminance > 0.0f ? mat.baseColor / luminance : splat(1.0f);
  float F0 = (1.0f - eta) / (1.0f + eta);
  specCol = mix(F0 * F0 * mix(splat(1.0f), ctint, mat.specularTint), mat.baseColor, mat.metallic);
  sheenCol = mix(splat(1.0f), ctint, mat.sheenTint);
}
RTD float GTR1(float NdotH, float alpha) {  // RT:431-436
  if (alpha >= 1) return INV_PI;
  float a2 = alpha * alpha;
  float t = 1 + (a2 - 1) * NdotH * NdotH;
  return (a2 - 1) / (PI * log_(a2) * t);
}
RTD float GTR2_Aniso(float NdotH, float HdotX, float HdotY, float ax, float ay) {  // RT:447-452
  float a = HdotX / ax;
  float b = HdotY / ay;
  float c = a * a + b * b + NdotH * NdotH;
  return 1.0f / (PI * ax * ay * c * c);
}
RTD float SmithG_GGX(float NdotV, float alphaG) {  // RT:456-461
  float a = alphaG * alphaG;
  float b = NdotV * NdotV;
  return (2.0f * NdotV) / (NdotV + sqrt_(a + b - a * b));
}
RTD float SmithG_GGX_Aniso(float NdotV, float VdotX, float VdotY, float ax, float ay) {  // RT:465-471
  float a = VdotX * ax;
  float b = VdotY * ay;
  float c = NdotV;
  return (2.0f * NdotV) / (NdotV + sqrt_(a * a + b * b + c * c));
}
RTD float SchlickFresnel(float u) {  // RT:475-479
  float m = clamp_(1.0f - u, 0.0f, 1.0f);
  float m2 = m * m;
  return m2 * m2 * m;
}
RTD float DielectricFresnel(float cosThetaI, float eta) {  // RT:483-497
  float sinThetaTSq = eta * eta * (1.0f - cosThetaI * cosThetaI);
  if (sinThetaTSq > 1.0f) return 1.0f;
  float cosThetaT = sqrt_(max_(1.0f - sinThetaTSq, 0.0f));
  float rs = (eta * cosThetaT - cosThetaI) / (eta * cosThetaT + cosThetaI);
  float rp = (eta * cosThetaI - cosThetaT) / (eta * cosThetaI + cosThetaT);
  return 0.5f * (rs * rs + rp * rp);
}
RTD float DisneyFresnel(const Mat& mat, float eta, float LDotH, float VDotH) {  // RT:501-506
  float metallicFresnel = SchlickFresnel(LDotH);
  float dielectricFresnel = DielectricFresnel(fabs_(VDotH), eta);
  return mix_(dielectricFresnel, metallicFresnel, mat.metallic);
}
RTD f3 ToWorld(f3 X, f3 Y, f3 Z, f3 V) { return V.x * X + V.y * Y + V.z * Z; }
RTD f3 ToLocal(f3 X, f3 Y, f3 Z, f3 V) { return mk3(dot(V, X), dot(V, Y), dot(V, Z)); }

RTD void CalculateBSDFLobePdfs(const Mat& material, f3 specCol, float approxFresnel, float& diffuseWeight,
                               float& specReflectWt, float& specRefractWt, float& clearcoatWt) {  // RT:537-550
  float lum = Luminance(material.baseColor);
  float r_diffuse = (1.0f - material.metallic) * (1.0f - material.transmission) * lum;
  float r_specular = Luminance(mix(specCol, splat(1.0f), approxFresnel));
  float r_clearcoat = (1.0f - material.metallic) * 0.25f * material.clearcoat;
  float r_refraction = (1.0f - material.metallic) * material.transmission * lum * (1.0f - approxFresnel);
  float r_sum_inv = 1.0f / (r_diffuse + r_specular + r_clearcoat + r_refraction);
  diffuseWeight = r_diffuse * r_sum_inv;
  specReflectWt = r_specular * r_sum_inv;
  clearcoatWt = r_clearcoat * r_sum_inv;
  specRefractWt = r_refraction * r_sum_inv;
}

RTD f3 CosineSampleHemisphere(float r1, float r2) {  // RT:650-659
  float r = sqrt_(r1);
  float phi = TWO_PI * r2;
  float s, c;
  sincos_(phi, &s, &c);
  f3 dir;
  dir.x = r * c;
  dir.y = r * s;
  dir.z = sqrt_(max_(0.0f, 1.0f - dir.x * dir.x - dir.y * dir.y));
  return dir;
}
RTD f3 SampleGTR1(float rgh, float r1) {  // RT:716-729 (R23: r1 used for both angles)
  float a = max_(0.001f, rgh);
  float a2 = a * a;
  float phi = r1 * TWO_PI;
  float cosTheta = sqrt_((1.0f - pow_(a2, 1.0f - r1)) / (1.0f - a2));
  float sinTheta = clamp_(sqrt_(1.0f - (cosTheta * cosTheta)), 0.0f, 1.0f);
  float sinPhi, cosPhi;
  sincos_(phi, &sinPhi, &cosPhi);
  return mk3(sinTheta * cosPhi, sinTheta * sinPhi, cosTheta);
}
// PRE (vt != nullptr): the terms that depend on V and the material only, precomputed by
// v_terms (camera-hit records, rt_wavefront.h cam_rec): vt[0] = DisneySample's lobe weights,
// vt[1] = {FV, G1V, GccV, Vh.x}, vt[2] = {Vh.yz, T1.xy}, vt[3] = {T1.z, T2}
RTD void ggx_vndf_frame(f3 V, float ax, float ay, f3& Vh, f3& T1, f3& T2) {  // RT:753-756
  Vh = normalize(mk3(ax * V.x, ay * V.y, V.z));
  float lensq = Vh.x * Vh.x + Vh.y * Vh.y;
  T1 = lensq > 0 ? mk3(-Vh.y, Vh.x, 0) * inversesqrt_(lensq) : mk3(1, 0, 0);
  T2 = cross(Vh, T1);
}
template <bool PRE = false>
RTD f3 SampleGGXVNDF(f3 V, float ax, float ay, float r1, float r2, const float4* vt = nullptr) {  // RT:751-769
  f3 Vh, T1, T2;
  if constexpr (PRE) {
    const float4 q1 = vt[1], q2 = vt[2], q3 = vt[3];
    Vh = mk3(q1.w, q2.x, q2.y);
    T1 = mk3(q2.z, q2.w, q3.x);
    T2 = mk3(q3.y, q3.z, q3.w);
  } else {
    ggx_vndf_frame(V, ax, ay, Vh, T1, T2);
  }
  float r = sqrt_(r1);
  float phi = 2.0f * PI * r2;
  float s, c;
  sincos_(phi, &s, &c);
  float t1 = r * c;
  float t2 = r * s;
  float sm = 0.5f * (1.0f + Vh.z);
  t2 = (1.0f - sm) * sqrt_(1.0f - t1 * t1) + sm * t2;
  f3 Nh = t1 * T1 + t2 * T2 + sqrt_(max_(0.0f, 1.0f - t1 * t1 - t2 * t2)) * Vh;
  return normalize(mk3(ax * Nh.x, ay * Nh.y, max_(0.0f, Nh.z)));
}

template <bool PRE = false>
RTD f3 EvalDiffuse(const Mat& mat, f3 Csheen, f3 V, f3 L, f3 H, float& pdf, const float4* vt = nullptr) {  // RT:925-948
  pdf = 0.0f;
  if (L.z <= 0.0f) return splat(0.0f);
  float FL = SchlickFresnel(L.z);
  float FV = PRE ? vt[1].x : SchlickFresnel(V.z);
  float LH = dot(L, H);
  float FH = SchlickFresnel(LH);
  float Fd90 = 0.5f + 2.0f * LH * LH * mat.roughness;
  float Fd = mix_(1.0f, Fd90, FL) * mix_(1.0f, Fd90, FV);
  float Fss90 = LH * LH * mat.roughness;
  float Fss = mix_(1.0f, Fss90, FL) * mix_(1.0f, Fss90, FV);
  float ss = 1.25f * (Fss * (1.0f / (L.z + V.z) - 0.5f) + 0.5f);
  f3 Fsheen = FH * mat.sheen * Csheen;
  pdf = L.z * INV_PI;
  return (1.0f - mat.metallic) * (1.0f - mat.transmission) * (INV_PI * mix_(Fd, ss, mat.subsurface) * mat.baseColor + Fsheen);
}
template <bool PRE = false>
RTD f3 EvalSpecReflection(const Mat& mat, float eta, f3 specCol, f3 V, f3 L, f3 H, float& pdf,
                          const float4* vt = nullptr) {  // RT:950-964
  pdf = 0.0f;
  if (L.z <= 0.0f) return splat(0.0f);
  float FM = DisneyFresnel(mat, eta, dot(L, H), dot(V, H));
  f3 F = mix(specCol, splat(1.0f), FM);
  float D = GTR2_Aniso(H.z, H.x, H.y, mat.ax, mat.ay);
  float G1 = PRE ? vt[1].y : SmithG_GGX_Aniso(fabs_(V.z), V.x, V.y, mat.ax, mat.ay);
  float G2 = G1 * SmithG_GGX_Aniso(fabs_(L.z), L.x, L.y, mat.ax, mat.ay);
  pdf = G1 * D / (4.0f * V.z);
  return F * D * G2 / (4.0f * L.z * V.z);
}
template <bool PRE = false>
RTD f3 EvalSpecRefraction(const Mat& mat, float eta, f3 V, f3 L, f3 H, float& pdf, const float4* vt = nullptr) {  // RT:966-984
  pdf = 0.0f;
  if (L.z >= 0.0f) return mk3(1.0f, 0.0f, 0.0f);  // R26
  float VH = dot(V, H), LH = dot(L, H);
  float F = DielectricFresnel(fabs_(VH), eta);
  float D = GTR2_Aniso(H.z, H.x, H.y, mat.ax, mat.ay);
  float G1 = PRE ? vt[1].y : SmithG_GGX_Aniso(fabs_(V.z), V.x, V.y, mat.ax, mat.ay);
  float G2 = G1 * SmithG_GGX_Aniso(fabs_(L.z), L.x, L.y, mat.ax, mat.ay);
  float denom = LH + VH * eta;
  denom *= denom;
  float eta2 = eta * eta;
  float jacobian = fabs_(LH) / denom;
  pdf = G1 * max_(0.0f, VH) * D * jacobian / V.z;
  f3 sq = mk3(pow_(mat.baseColor.x, 0.5f), pow_(mat.baseColor.y, 0.5f), pow_(mat.baseColor.z, 0.5f));
  return sq * (1.0f - mat.metallic) * mat.transmission * (1.0f - F) * D * G2 * fabs_(VH) * jacobian * eta2 /
         fabs_(L.z * V.z);
}
template <bool PRE = false>
RTD f3 EvalClearcoat(const Mat& mat, f3 V, f3 L, f3 H, float& pdf, const float4* vt = nullptr) {  // RT:986-1000 (R23)
  pdf = 0.0f;
  if (L.z <= 0.0f) return splat(0.0f);
  float VH = dot(V, H);
  float FH = DielectricFresnel(VH, 1.0f / 1.5f);
  float F = mix_(0.04f, 1.0f, FH);
  float D = GTR1(H.z, mat.clearcoatGloss);
  float G = SmithG_GGX(L.z, 0.25f) * (PRE ? vt[1].z : SmithG_GGX(V.z, 0.25f));
  float jacobian = 1.0f / (4.0f * VH);
  pdf = D * H.z * jacobian;
  return splat(0.25f) * mat.clearcoat * F * D * G / (4.0f * L.z * V.z);
}

// The part of DisneyEval / DisneySample that depends only on (material, V, N): one bounce's
// NEE evaluation, BSDF sample and continuation evaluation share it (same operations, computed
// once instead of three times).
struct BsdfFrame {
  float eta;
  f3 T, B, V;  // tangent frame of N (RT:396-407) and V in it
  f3 specCol, sheenCol;
};
RTD BsdfFrame bsdf_frame(const Mat& material, f3 V, f3 N) {
  BsdfFrame F;
  F.eta = dot(V, N) > 0.0f ? (1.0f / material.IOR) : material.IOR;  // R10 (RT:1010, RT:1079)
  getTangent(N, F.T, F.B);
  F.V = ToLocal(F.T, F.B, N, V);
  GetSpecColor(material, F.eta, F.specCol, F.sheenCol);
  return F;
}
// DisneySample's lobe weights (RT:1083-1084): from the Fresnel term at V.z alone
RTD void sample_lobe_wts(const BsdfFrame& F, const Mat& material, float& diffuseWt, float& specReflectWt,
                         float& specRefractWt, float& clearcoatWt) {
  float approxFresnel = DisneyFresnel(material, F.eta, F.V.z, F.V.z);
  CalculateBSDFLobePdfs(material, F.specCol, approxFresnel, diffuseWt, specReflectWt, specRefractWt, clearcoatWt);
}
// the V-only terms of the PRE variants (layout above SampleGGXVNDF), the same operations
RTD void v_terms(const BsdfFrame& F, const Mat& m, float4* vt) {
  const f3 V = F.V;
  float dW, sRW, sTW, cW;
  sample_lobe_wts(F, m, dW, sRW, sTW, cW);
  f3 Vh, T1, T2;
  ggx_vndf_frame(V, m.ax, m.ay, Vh, T1, T2);
  vt[0] = make_float4(dW, sRW, sTW, cW);
  vt[1] = make_float4(SchlickFresnel(V.z), SmithG_GGX_Aniso(fabs_(V.z), V.x, V.y, m.ax, m.ay), SmithG_GGX(V.z, 0.25f), Vh.x);
  vt[2] = make_float4(Vh.y, Vh.z, T1.x, T1.y);
  vt[3] = make_float4(T1.z, T2.x, T2.y, T2.z);
}

template <bool PRE = false>
RTD f3 DisneyEval(const BsdfFrame& F, const Mat& material, f3 N, f3 L, float& bsdfPdf,
                  const float4* vt = nullptr) {  // RT:1002-1067
  bsdfPdf = 0.0f;
  f3 f = splat(0.0f);
  const float eta = F.eta;
  const f3 T = F.T, B = F.B, V = F.V;
  L = ToLocal(T, B, N, L);
  f3 H;
  if (L.z > 0.0f) H = normalize(L + V);
  else H = normalize(L + V * eta);
  if (H.z < 0.0f) H = -H;
  const f3 specCol = F.specCol, sheenCol = F.sheenCol;
  float diffuseWt, specReflectWt, specRefractWt, clearcoatWt;
  float fresnel = DisneyFresnel(material, eta, dot(L, H), dot(V, H));
  CalculateBSDFLobePdfs(material, specCol, fresnel, diffuseWt, specReflectWt, specRefractWt, clearcoatWt);
  float pdf;
  if (diffuseWt > 0.0f && L.z > 0.0f) {
    f = f + EvalDiffuse<PRE>(material, sheenCol, V, L, H, pdf, vt);
    bsdfPdf += pdf * diffuseWt;
  }
  if (specReflectWt > 0.0f && L.z > 0.0f && V.z > 0.0f) {
    f = f + EvalSpecReflection<PRE>(material, eta, specCol, V, L, H, pdf, vt);
    bsdfPdf += pdf * specReflectWt;
  }
  if (specRefractWt > 0.0f && L.z < 0.0f) {
    f = f + EvalSpecRefraction<PRE>(material, eta, V, L, H, pdf, vt);
    bsdfPdf += pdf * specRefractWt;
  }
  if (clearcoatWt > 0.0f && L.z > 0.0f && V.z > 0.0f) {
    f = f + EvalClearcoat<PRE>(material, V, L, H, pdf, vt);
    bsdfPdf += pdf * clearcoatWt;
  }
  return f * fabs_(L.z);
}
RTD f3 DisneyEval(const Mat& material, f3 V, f3 N, f3 L, float& bsdfPdf) {
  return DisneyEval(bsdf_frame(material, V, N), material, N, L, bsdfPdf);
}

template <bool PRE = false>
RTD f3 DisneySample(const BsdfFrame& F, float xi_1, float xi_2, float xi_3, const Mat& material, f3 N, f3& L,
                    float& pdf, bool& isRefract, const float4* vt = nullptr) {  // RT:1070-1161
  pdf = 0.0f;
  f3 f = splat(0.0f);
  isRefract = false;
  float r1 = xi_1;
  float r2 = xi_2;
  const float eta = F.eta;
  const f3 T = F.T, B = F.B, V = F.V;
  const f3 specCol = F.specCol, sheenCol = F.sheenCol;
  float diffuseWt, specReflectWt, specRefractWt, clearcoatWt;
  if constexpr (PRE) {
    const float4 q0 = vt[0];
    diffuseWt = q0.x; specReflectWt = q0.y; specRefractWt = q0.z; clearcoatWt = q0.w;
  } else {
    sample_lobe_wts(F, material, diffuseWt, specReflectWt, specRefractWt, clearcoatWt);
  }
  float cdf0 = diffuseWt;
  float cdf1 = cdf0 + clearcoatWt;
  L = splat(0.0f);  // R7
  if (r1 < cdf0) {
    r1 /= cdf0;
    L = CosineSampleHemisphere(r1, r2);
    f3 H = normalize(L + V);
    f = EvalDiffuse<PRE>(material, sheenCol, V, L, H, pdf, vt);
    pdf *= diffuseWt;
  } else if (r1 < cdf1) {
    r1 = (r1 - cdf0) / (cdf1 - cdf0);
    f3 H = SampleGTR1(material.clearcoatGloss, r1);
    if (H.z < 0.0f) H = -H;
    L = normalize(reflect(-V, H));
    f = EvalClearcoat<PRE>(material, V, L, H, pdf, vt);
    pdf *= clearcoatWt;
  } else {
    r1 = (r1 - cdf1) / (1.0f - cdf1);
    f3 H = SampleGGXVNDF<PRE>(V, material.ax, material.ay, r1, r2, vt);
    if (H.z < 0.0f) H = -H;
    float fresnel = DisneyFresnel(material, eta, dot(L, H), dot(V, H));  // R7: L == 0 here
    float F = 1.0f - ((1.0f - fresnel) * material.transmission * (1.0f - material.metallic));
    if (xi_3 < F) {
      L = normalize(reflect(-V, H));
      f = EvalSpecReflection<PRE>(material, eta, specCol, V, L, H, pdf, vt);
      pdf *= F;
    } else {
      isRefract = true;
      L = normalize(refract(-V, H, eta));  // R14
      f = EvalSpecRefraction<PRE>(material, eta, V, L, H, pdf, vt);
      pdf *= (1.0f - F);
    }
    pdf *= specReflectWt + specRefractWt;
  }
  L = ToWorld(T, B, N, L);
  return f * fabs_(dot(N, L));
}
RTD f3 DisneySample(float xi_1, float xi_2, float xi_3, const Mat& material, f3 V, f3 N, f3& L, float& pdf,
                    bool& isRefract) {
  return DisneySample(bsdf_frame(material, V, N), xi_1, xi_2, xi_3, material, N, L, pdf, isRefract);
}

// ----------------------------------------------------------- BRDF mode (enableBSDF == false)
RTD float GTR2(float NdotH, float alpha) {  // RT:441-445
  float a2 = alpha * alpha;
  float t = 1 + (a2 - 1) * NdotH * NdotH;
  return a2 / (PI * t * t);
}
RTD void CalculateBRDFLobePdfs(const Mat& m, float& pDiffuse, float& pSpecular, float& pClearcoat) {  // RT:520-533
  float r_diffuse = (1.0f - m.metallic);
  float r_specular = (1.0f - m.metallic) + m.metallic;
  float r_clearcoat = (1.0f - m.metallic) * 0.25f * m.clearcoat;
  float r_sum_inv = 1.0f / (r_diffuse + r_specular + r_clearcoat);
  pDiffuse = r_diffuse * r_sum_inv;
  pSpecular = r_specular * r_sum_inv;
  pClearcoat = r_clearcoat * r_sum_inv;
}
RTD f3 toNormalHemisphere(f3 v, f3 N) {  // RT:663-669
  f3 helper = mk3(1, 0, 0);
  if (fabs_(N.x) > 0.999f) helper = mk3(0, 0, 1);
  f3 tangent = normalize(cross(N, helper));
  f3 bitangent = normalize(cross(N, tangent));
  return v.x * tangent + v.y * bitangent + v.z * N;
}
RTD f3 SampleCosineHemisphere(float xi_1, float xi_2, f3 N) {  // RT:673-685
  float r = sqrt_(xi_1);
  float theta = xi_2 * TWO_PI;
  float x = r * cos_(theta);
  float y = r * sin_(theta);
  float z = sqrt_(1.0f - x * x - y * y);
  return toNormalHemisphere(mk3(x, y, z), N);
}
RTD f3 SampleGTR1_h(float xi_1, float xi_2, f3 V, f3 N, float alpha) {  // RT:697-714
  float phi_h = xi_1 * TWO_PI;
  float sin_phi_h = sin_(phi_h);
  float cos_phi_h = cos_(phi_h);
  float cos_theta_h = sqrt_((1.0f - pow_(alpha * alpha, 1.0f - xi_2)) / (1.0f - alpha * alpha));
  float sin_theta_h = sqrt_(max_(0.0f, 1.0f - cos_theta_h * cos_theta_h));
  f3 H = mk3(sin_theta_h * cos_phi_h, sin_theta_h * sin_phi_h, cos_theta_h);
  H = toNormalHemisphere(H, N);
  return reflect(-V, H);
}
RTD f3 SampleGTR2(float xi_1, float xi_2, f3 V, f3 N, float alpha) {  // RT:732-749
  float phi_h = 2.0f * PI * xi_1;
  float sin_phi_h = sin_(phi_h);
  float cos_phi_h = cos_(phi_h);
  float cos_theta_h = sqrt_((1.0f - xi_2) / (1.0f + (alpha * alpha - 1.0f) * xi_2));
  float sin_theta_h = sqrt_(max_(0.0f, 1.0f - cos_theta_h * cos_theta_h));
  f3 H = mk3(sin_theta_h * cos_phi_h, sin_theta_h * sin_phi_h, cos_theta_h);
  H = toNormalHemisphere(H, N);
  return reflect(-V, H);
}
RTD f3 SampleBRDF(float xi_1, float xi_2, float xi_3, f3 V, f3 N, const Mat& m) {  // RT:789-833
  float p_diffuse, p_specular, p_clearcoat;
  CalculateBRDFLobePdfs(m, p_diffuse, p_specular, p_clearcoat);
  float alpha_GTR1 = mix_(0.1f, 0.001f, m.clearcoatGloss);
  float alpha_GTR2 = max_(0.001f, sqr(m.roughness));
  float cdf0 = p_diffuse;
  float cdf1 = cdf0 + p_clearcoat;
  float cdf2 = cdf1 + p_specular;
  // RT:808-817 compute an eta, a VNDF half vector and a Fresnel that are never used
  if (xi_3 <= cdf0) return SampleCosineHemisphere(xi_1, xi_2, N);
  else if (xi_3 <= cdf1) return SampleGTR1_h(xi_1, xi_2, V, N, alpha_GTR1);
  else if (xi_3 <= cdf2) return SampleGTR2(xi_1, xi_2, V, N, alpha_GTR2);
  return mk3(0, 1, 0);
}
RTD f3 BRDF_Evaluate(f3 V, f3 N, f3 L, f3 X, f3 Y, const Mat& m, float& pdf) {  // RT:836-921
  pdf = 1e-10f;
  float NdotL = dot(N, L);
  float NdotV = dot(N, V);
  if (NdotL < 0 || NdotV < 0) return splat(0.0f);
  f3 H = normalize(L + V);
  float NdotH = dot(N, H);
  float LdotH = dot(L, H);
  f3 Cdlin = m.baseColor;
  float Cdlum = Luminance(Cdlin);
  f3 Ctint = (Cdlum > 0) ? (Cdlin / Cdlum) : splat(1.0f);
  f3 Cspec = m.specular * mix(splat(1.0f), Ctint, m.specularTint);
  f3 Cspec0 = mix(0.08f * Cspec, Cdlin, m.metallic);
  f3 Csheen = mix(splat(1.0f), Ctint, m.sheenTint);
  float Fd90 = 0.5f + 2.0f * LdotH * LdotH * m.roughness;
  float FL = SchlickFresnel(NdotL);
  float FV = SchlickFresnel(NdotV);
  float Fd = mix_(1.0f, Fd90, FL) * mix_(1.0f, Fd90, FV);
  float Fss90 = LdotH * LdotH * m.roughness;
  float Fss = mix_(1.0f, Fss90, FL) * mix_(1.0f, Fss90, FV);
  float ss = 1.25f * (Fss * (1.0f / (NdotL + NdotV) - 0.5f) + 0.5f);
  float FH = SchlickFresnel(LdotH);
  float alpha = max_(0.001f, sqr(m.roughness));
  float Ds = GTR2(NdotH, alpha);
  f3 Fs = mix(Cspec0, splat(1.0f), FH);
  float Gs = SmithG_GGX(NdotL, m.roughness);  // R27: roughness, not alpha
  Gs *= SmithG_GGX(NdotV, m.roughness);
  if (m.anisotropic > 0) {
    Ds = GTR2_Aniso(NdotH, dot(H, X), dot(H, Y), m.ax, m.ay);
    Gs = SmithG_GGX_Aniso(NdotL, dot(L, X), dot(L, Y), m.ax, m.ay);
    Gs *= SmithG_GGX_Aniso(NdotV, dot(V, X), dot(V, Y), m.ax, m.ay);
  }
  float Dr = GTR1(NdotH, mix_(0.1f, 0.001f, 1.0f - m.clearcoatGloss));
  float Fr = mix_(0.04f, 1.0f, FH);
  float Gr = SmithG_GGX(NdotL, 0.25f) * SmithG_GGX(NdotV, 0.25f);
  f3 Fsheen = FH * m.sheen * Csheen;
  f3 diffuse = INV_PI * mix_(Fd, ss, m.subsurface) * Cdlin + Fsheen;
  f3 specular = Gs * Fs * Ds / (4.0f * NdotV * NdotL);
  f3 clearcoat = splat(0.25f) * Gr * Fr * Dr * m.clearcoat / (4.0f * NdotV * NdotL);
  float p_diffuse, p_specular, p_clearcoat;
  CalculateBRDFLobePdfs(m, p_diffuse, p_specular, p_clearcoat);
  float pdf_diffuse = NdotL * INV_PI;
  float pdf_specular = Ds * NdotH / (4.0f * LdotH);
  float pdf_clearcoat = Dr * NdotH / (4.0f * LdotH);
  pdf = p_diffuse * pdf_diffuse + p_specular * pdf_specular + p_clearcoat * pdf_clearcoat;
  pdf = max_(1e-10f, pdf);
  return (1.0f - m.metallic) * diffuse + specular + clearcoat;
}

RTD f3 SampleHG(f3 V, float g, float r1, float r2) {  // RT:1195-1216
  float cosTheta;
  if (fabs_(g) < 0.001f) cosTheta = 1 - 2 * r2;
  else {
    float sqrTerm = (1 - g * g) / (1 + g - 2 * g * r2);
    cosTheta = -(1 + g * g - sqrTerm * sqrTerm) / (2 * g);
  }
  float phi = r1 * TWO_PI;
  float sinTheta = clamp_(sqrt_(1.0f - (cosTheta * cosTheta)), 0.0f, 1.0f);
  float sinPhi, cosPhi;
  sincos_(phi, &sinPhi, &cosPhi);
  f3 v1, v2;
  getTangent(V, v1, v2);
  return sinTheta * cosPhi * v1 + sinTheta * sinPhi * v2 + cosTheta * V;
}
RTD float PhaseHG(float cosTheta, float g) {  // RT:1218-1222
  float denom = 1 + g * g + 2 * g * cosTheta;
  return INV_4_PI * (1 - g * g) / (denom * sqrt_(denom));
}
RTD float misMixWeight(float a, float b) {  // RT:1285-1288
  float t = a * a;
  return t / (b * b + t);
}

}  // namespace rtd
