// oracle/rt_oracle.cpp — TEST INFRASTRUCTURE ONLY (never linked into the product).
//
// A literal CPU restatement of the reference per-pixel path tracer
//   /root/reference/src/shaders/fragment_shader_ray_tracing.glsl   ("RT:<line>")
// driven the way src/sources/main.cpp:175-200 drives it (one fragment per pixel,
// TexCoords = ((px+0.5)/W, (py+0.5)/H) from src/shaders/vertex_shader.glsl and the
// full-screen quad of src/core/Screen.h:8-16).  Inputs are the reference's own GPU
// encodings: Triangle_encoded (14 x vec3, src/core/Triangle.h:28-39) and
// BVHNode_encoded (4 x vec3, src/core/BVH.h:17-21), the RGB32F HDR map and the
// hdrCache texture (src/core/Utility.h:33-131).
//
// Allowed users: tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
//
// Parity status: the GLSL program cannot execute in this container (no GL
// context), so this restatement is NOT pinned against reference
// output images ("parity unpinned" at image level).  Its inputs are pinned:
// the HDR decode against the reference hdrloader built from its own sources
// (oracle/_ref), the BVH topology against node/leaf/depth counts measured from
// the reference BVH.h, plus hand-derived known answers
// (tests/test_oracle_kat.py).  GLSL builtins are evaluated with the deterministic
// definitions in glsl_math.h; the quirks R1-R28 of SURVEY.md §8(a) are mirrored
// and marked "R<n>" below.
//
// Build: oracle/Makefile (g++ -O2 -ffp-contract=off -fopenmp).
#include <stdint.h>
#include <string.h>
#include <math.h>
#include "../opengl-ray-tracing-framework_amd/csrc/common/glsl_math.h"
#ifdef _OPENMP
#include <omp.h>
#endif

using namespace gm;

namespace {

// ----------------------------------------------------------------------------- vec
struct vec2 { float x, y; };
struct vec3 {
  float x, y, z;
  vec3() : x(0), y(0), z(0) {}
  vec3(float a) : x(a), y(a), z(a) {}
  vec3(float a, float b, float c) : x(a), y(b), z(c) {}
};
inline vec3 operator+(vec3 a, vec3 b) { return vec3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline vec3 operator-(vec3 a, vec3 b) { return vec3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline vec3 operator*(vec3 a, vec3 b) { return vec3(a.x * b.x, a.y * b.y, a.z * b.z); }
inline vec3 operator/(vec3 a, vec3 b) { return vec3(a.x / b.x, a.y / b.y, a.z / b.z); }
inline vec3 operator*(vec3 a, float s) { return vec3(a.x * s, a.y * s, a.z * s); }
inline vec3 operator*(float s, vec3 a) { return vec3(s * a.x, s * a.y, s * a.z); }
inline vec3 operator/(vec3 a, float s) { return vec3(a.x / s, a.y / s, a.z / s); }
inline vec3 operator-(vec3 a) { return vec3(-a.x, -a.y, -a.z); }
inline float dot(vec3 a, vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline vec3 cross(vec3 a, vec3 b) {
  return vec3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
inline vec3 normalize(vec3 v) { float inv = 1.0f / sqrt_(dot(v, v)); return v * inv; }
inline vec3 vmin(vec3 a, vec3 b) { return vec3(min_(a.x, b.x), min_(a.y, b.y), min_(a.z, b.z)); }
inline vec3 vmax(vec3 a, vec3 b) { return vec3(max_(a.x, b.x), max_(a.y, b.y), max_(a.z, b.z)); }
inline vec3 mix(vec3 x, vec3 y, float a) { return x * (1.0f - a) + y * a; }
inline vec3 exp3(vec3 v) { return vec3(exp_(v.x), exp_(v.y), exp_(v.z)); }
inline vec3 pow3(vec3 v, vec3 e) { return vec3(pow_(v.x, e.x), pow_(v.y, e.y), pow_(v.z, e.z)); }
// GLSL reflect/refract (GLSL 4.50 §8.5)
inline vec3 reflect(vec3 I, vec3 N) { return I - 2.0f * dot(N, I) * N; }
inline vec3 refract(vec3 I, vec3 N, float eta) {
  float k = 1.0f - eta * eta * (1.0f - dot(N, I) * dot(N, I));
  if (k < 0.0f) return vec3(0.0f);
  return eta * I - (eta * dot(N, I) + sqrt_(k)) * N;
}

const float PI = 3.14159265358979323f;
const float INV_PI = 0.31830988618379067f;
const float TWO_PI = 6.28318530717958648f;
const float INV_4_PI = 0.07957747154594766f;
const float EPS = 0.0001f;
const float INF = 114514.0f;
const int SIZE_TRIANGLE = 14;
const int SIZE_BVHNODE = 4;
const int MEDIUM_ABSORB = 1, MEDIUM_SCATTER = 2, MEDIUM_EMISSIVE = 3;

}  // namespace

// ------------------------------------------------------------------------- C-ABI types
extern "C" {
typedef struct {
  const float* triangles;  // n_triangles * 14 * 3 floats (Triangle_encoded)
  int n_triangles;
  const float* nodes;      // n_nodes * 4 * 3 floats (BVHNode_encoded), node 0 = dummy
  int n_nodes;
  const float* hdr_map;    // hdr_w * hdr_h * 3 (row 0 = first uploaded row)
  const float* hdr_cache;  // hdr_w * hdr_h * 3 (x, y, pdf)
  int hdr_w, hdr_h;
  int hdr_resolution;      // uniform hdrResolution (= hdr_w, src/core/Scene.h:183)
} orc_scene;

typedef struct {  // the per-frame uniforms of src/sources/main.cpp:181-199
  float position[3], front[3], right[3], up[3], left_bottom_corner[3];
  float half_h, half_w;
  int loop_num;
  float rand_origin;
  int enable_mis, enable_env_map, enable_bsdf;
  float env_intensity, env_angle;
  int max_bounce, max_iterations;
} orc_frame;

typedef struct {  // traversal counters for SURVEY.md §8(d)
  uint64_t rays, internal_pops, leaf_pops, tri_tests, closer_updates, samples, env_fetches, cache_fetches;
} orc_counters;
}

namespace {

// ------------------------------------------------------------------ structs RT:22-101
struct Triangle { vec3 p1, p2, p3, n1, n2, n3; };
struct BVHNode { int left, right, n, index; vec3 AA, BB; };
struct Medium { int type; float density; vec3 color; float anisotropy; };
struct Material {
  vec3 emissive, baseColor;
  float subsurface, metallic, specular, specularTint, roughness, anisotropic, sheen, sheenTint,
      clearcoat, clearcoatGloss, IOR, transmission, ax, ay;
  Medium medium;
};
struct Ray { vec3 origin, direction; };
struct HitRecord {
  bool isHit, isInside;
  vec3 hitPoint, normal, viewDir;
  float distance;
  Material material;
};

struct Ctx {  // "uniforms" + per-invocation globals (wseed RT:573) + counters
  const orc_scene* s;
  const orc_frame* f;
  uint32_t wseed;
  orc_counters c;
};

// texelFetch on a samplerBuffer: out-of-range texels read as 0 (robust access)
inline vec3 texelTri(const Ctx& C, int i) {
  if (i < 0 || i >= C.s->n_triangles * SIZE_TRIANGLE) return vec3(0.0f);
  const float* p = C.s->triangles + 3 * (size_t)i;
  return vec3(p[0], p[1], p[2]);
}
inline vec3 texelNode(const Ctx& C, int i) {
  if (i < 0 || i >= C.s->n_nodes * SIZE_BVHNODE) return vec3(0.0f);
  const float* p = C.s->nodes + 3 * (size_t)i;
  return vec3(p[0], p[1], p[2]);
}
// texture() on the RGB32F hdrMap/hdrCache: NEAREST + CLAMP_TO_EDGE (src/core/Model.h:241-245), R13
inline vec3 tex2D(const float* img, int w, int h, vec2 uv) {
  int i = (int)floor_(uv.x * (float)w);
  int j = (int)floor_(uv.y * (float)h);
  if (isnan_(uv.x)) i = 0;
  if (isnan_(uv.y)) j = 0;
  if (i < 0) i = 0;
  if (i > w - 1) i = w - 1;
  if (j < 0) j = 0;
  if (j > h - 1) j = h - 1;
  const float* p = img + 3 * ((size_t)j * w + i);
  return vec3(p[0], p[1], p[2]);
}

inline float sqr(float x) { return x * x; }                                      // RT:138
inline float Luminance(vec3 c) { return 0.212671f * c.x + 0.715160f * c.y + 0.072169f * c.z; }  // RT:142

Triangle getTriangle(const Ctx& C, int i) {  // RT:149-164
  int offset = i * SIZE_TRIANGLE;
  Triangle t;
  t.p1 = texelTri(C, offset + 0); t.p2 = texelTri(C, offset + 1); t.p3 = texelTri(C, offset + 2);
  t.n1 = texelTri(C, offset + 3); t.n2 = texelTri(C, offset + 4); t.n3 = texelTri(C, offset + 5);
  return t;
}

Material getMaterial(const Ctx& C, int i) {  // RT:174-214
  Material m;
  int offset = i * SIZE_TRIANGLE;
  vec3 param1 = texelTri(C, offset + 8);
  vec3 param2 = texelTri(C, offset + 9);
  vec3 param3 = texelTri(C, offset + 10);
  vec3 param4 = texelTri(C, offset + 11);
  vec3 param5 = texelTri(C, offset + 13);
  m.emissive = texelTri(C, offset + 6);
  m.baseColor = texelTri(C, offset + 7);
  m.medium.color = texelTri(C, offset + 12);
  m.subsurface = param1.x; m.metallic = param1.y; m.specular = param1.z;
  m.specularTint = param2.x; m.roughness = param2.y; m.anisotropic = param2.z;
  m.sheen = param3.x; m.sheenTint = param3.y; m.clearcoat = param3.z;
  m.clearcoatGloss = param4.x; m.IOR = param4.y; m.transmission = param4.z;
  float aspect = sqrt_(1.0f - m.anisotropic * 0.9f);
  m.ax = max_(0.001f, sqr(m.roughness) / aspect);
  m.ay = max_(0.001f, sqr(m.roughness) * aspect);
  m.medium.type = (int)param5.x;
  m.medium.density = param5.y;
  m.medium.anisotropy = param5.z;
  return m;
}

BVHNode getBVHNode(const Ctx& C, int i) {  // RT:218-237
  BVHNode node;
  int offset = i * SIZE_BVHNODE;
  vec3 childs = texelNode(C, offset + 0);
  vec3 leafInfo = texelNode(C, offset + 1);
  node.left = (int)childs.x; node.right = (int)childs.y;
  node.n = (int)leafInfo.x; node.index = (int)leafInfo.y;
  node.AA = texelNode(C, offset + 2);
  node.BB = texelNode(C, offset + 3);
  return node;
}

HitRecord hitTriangle(Triangle triangle, Ray ray) {  // RT:241-299 (R1: plane + edge test)
  HitRecord rec;
  rec.distance = INF; rec.isHit = false; rec.isInside = false;
  vec3 p1 = triangle.p1, p2 = triangle.p2, p3 = triangle.p3;
  vec3 S = ray.origin, d = ray.direction;
  vec3 N = normalize(cross(p2 - p1, p3 - p1));
  if (dot(N, d) > 0.0f) { N = -N; rec.isInside = true; }
  if (fabs_(dot(N, d)) < 0.00001f) return rec;
  float t = (dot(N, p1) - dot(S, N)) / dot(d, N);
  if (t < 0.0005f) return rec;
  vec3 P = S + d * t;
  vec3 c1 = cross(p2 - p1, P - p1);
  vec3 c2 = cross(p3 - p2, P - p2);
  vec3 c3 = cross(p1 - p3, P - p3);
  bool r1 = (dot(c1, N) > 0 && dot(c2, N) > 0 && dot(c3, N) > 0);
  bool r2 = (dot(c1, N) < 0 && dot(c2, N) < 0 && dot(c3, N) < 0);
  if (r1 || r2) {
    rec.isHit = true;
    rec.hitPoint = P;
    rec.distance = t - 0.00001f;
    rec.viewDir = d;
    rec.normal = N;
    // R22: xy-projected barycentrics with +1e-7 in the denominators
    float alpha = (-(P.x - p2.x) * (p3.y - p2.y) + (P.y - p2.y) * (p3.x - p2.x)) /
                  (-(p1.x - p2.x) * (p3.y - p2.y) + (p1.y - p2.y) * (p3.x - p2.x) + 1e-7f);
    float beta = (-(P.x - p3.x) * (p1.y - p3.y) + (P.y - p3.y) * (p1.x - p3.x)) /
                 (-(p2.x - p3.x) * (p1.y - p3.y) + (p2.y - p3.y) * (p1.x - p3.x) + 1e-7f);
    float gama = 1.0f - alpha - beta;
    vec3 Nsmooth = alpha * triangle.n1 + beta * triangle.n2 + gama * triangle.n3;
    Nsmooth = normalize(Nsmooth);
    rec.normal = rec.isInside ? (-Nsmooth) : Nsmooth;
  }
  return rec;
}

float hitAABB(Ray r, vec3 AA, vec3 BB) {  // RT:303-316
  vec3 invdir = vec3(1.0f) / r.direction;
  vec3 f = (BB - r.origin) * invdir;
  vec3 n = (AA - r.origin) * invdir;
  vec3 tmax = vmax(f, n);
  vec3 tmin = vmin(f, n);
  float t1 = min_(tmax.x, min_(tmax.y, tmax.z));
  float t0 = max_(tmin.x, max_(tmin.y, tmin.z));
  return (t1 >= t0) ? ((t0 > 0.0f) ? t0 : t1) : -1.0f;
}

HitRecord hitArray(Ctx& C, Ray ray, int l, int r) {  // RT:320-334
  HitRecord rec;
  rec.isHit = false; rec.distance = INF;
  for (int i = l; i <= r; i++) {
    Triangle triangle = getTriangle(C, i);
    C.c.tri_tests++;
    HitRecord rr = hitTriangle(triangle, ray);
    if (rr.isHit && rr.distance < rec.distance) {
      rec = rr;
      rec.material = getMaterial(C, i);
      C.c.closer_updates++;
    }
  }
  return rec;
}

HitRecord hitBVH(Ctx& C, Ray ray) {  // RT:338-392 (R2: no closest-hit culling; R3 stack 256; R4 root 1)
  C.c.rays++;
  HitRecord rec;
  rec.isHit = false; rec.distance = INF;
  int stack[256];
  int sp = 0;
  stack[sp++] = 1;
  while (sp > 0) {
    int top = stack[--sp];
    BVHNode node = getBVHNode(C, top);
    if (node.n > 0) {
      C.c.leaf_pops++;
      int L = node.index;
      int R = node.index + node.n - 1;
      HitRecord r = hitArray(C, ray, L, R);
      if (r.isHit && r.distance < rec.distance) rec = r;
      continue;
    }
    C.c.internal_pops++;
    float d1 = INF, d2 = INF;
    if (node.left > 0) { BVHNode leftNode = getBVHNode(C, node.left); d1 = hitAABB(ray, leftNode.AA, leftNode.BB); }
    if (node.right > 0) { BVHNode rightNode = getBVHNode(C, node.right); d2 = hitAABB(ray, rightNode.AA, rightNode.BB); }
    if (d1 > 0 && d2 > 0) {
      if (d1 < d2) { stack[sp++] = node.right; stack[sp++] = node.left; }
      else { stack[sp++] = node.left; stack[sp++] = node.right; }
    } else if (d1 > 0) {
      stack[sp++] = node.left;
    } else if (d2 > 0) {
      stack[sp++] = node.right;
    }
    if (sp > 254) break;  // R3: the GLSL stack is unchecked; never reached (depth <= 64)
  }
  return rec;
}

void getTangent(vec3 N, vec3& tangent, vec3& bitangent) {  // RT:396-407
  vec3 helper = vec3(1, 0, 0);
  if (fabs_(N.x) > 0.999f) helper = vec3(0, 0, 1);
  bitangent = normalize(cross(N, helper));
  tangent = normalize(cross(N, bitangent));
}

void GetSpecColor(const Material& mat, float eta, vec3& specCol, vec3& sheenCol) {  // RT:420-427
  float luminance = Luminance(mat.baseColor);
  vec3 ctint = luminance > 0.0f ? mat.baseColor / luminance : vec3(1.0f);
  float F0 = (1.0f - eta) / (1.0f + eta);
  specCol = mix(F0 * F0 * mix(vec3(1.0f), ctint, mat.specularTint), mat.baseColor, mat.metallic);
  sheenCol = mix(vec3(1.0f), ctint, mat.sheenTint);
}

float GTR1(float NdotH, float alpha) {  // RT:431-436
  if (alpha >= 1) return INV_PI;
  float a2 = alpha * alpha;
  float t = 1 + (a2 - 1) * NdotH * NdotH;
  return (a2 - 1) / (PI * log_(a2) * t);
}
float GTR2(float NdotH, float alpha) {  // RT:441-445
  float a2 = alpha * alpha;
  float t = 1 + (a2 - 1) * NdotH * NdotH;
  return a2 / (PI * t * t);
}
float GTR2_Aniso(float NdotH, float HdotX, float HdotY, float ax, float ay) {  // RT:447-452
  float a = HdotX / ax;
  float b = HdotY / ay;
  float c = a * a + b * b + NdotH * NdotH;
  return 1.0f / (PI * ax * ay * c * c);
}
float SmithG_GGX(float NdotV, float alphaG) {  // RT:456-461
  float a = alphaG * alphaG;
  float b = NdotV * NdotV;
  return (2.0f * NdotV) / (NdotV + sqrt_(a + b - a * b));
}
float SmithG_GGX_Aniso(float NdotV, float VdotX, float VdotY, float ax, float ay) {  // RT:465-471
  float a = VdotX * ax;
  float b = VdotY * ay;
  float c = NdotV;
  return (2.0f * NdotV) / (NdotV + sqrt_(a * a + b * b + c * c));
}
float SchlickFresnel(float u) {  // RT:475-479
  float m = clamp_(1.0f - u, 0.0f, 1.0f);
  float m2 = m * m;
  return m2 * m2 * m;
}
float DielectricFresnel(float cosThetaI, float eta) {  // RT:483-497
  float sinThetaTSq = eta * eta * (1.0f - cosThetaI * cosThetaI);
  if (sinThetaTSq > 1.0f) return 1.0f;
  float cosThetaT = sqrt_(max_(1.0f - sinThetaTSq, 0.0f));
  float rs = (eta * cosThetaT - cosThetaI) / (eta * cosThetaT + cosThetaI);
  float rp = (eta * cosThetaI - cosThetaT) / (eta * cosThetaI + cosThetaT);
  return 0.5f * (rs * rs + rp * rp);
}
float DisneyFresnel(const Material& mat, float eta, float LDotH, float VDotH) {  // RT:501-506
  float metallicFresnel = SchlickFresnel(LDotH);
  float dielectricFresnel = DielectricFresnel(fabs_(VDotH), eta);
  return mix_(dielectricFresnel, metallicFresnel, mat.metallic);
}
vec3 ToWorld(vec3 X, vec3 Y, vec3 Z, vec3 V) { return V.x * X + V.y * Y + V.z * Z; }    // RT:508
vec3 ToLocal(vec3 X, vec3 Y, vec3 Z, vec3 V) { return vec3(dot(V, X), dot(V, Y), dot(V, Z)); }  // RT:513

void CalculateBSDFLobePdfs(const Material& material, float eta, vec3 specCol, float approxFresnel,
                           float& diffuseWeight, float& specReflectWt, float& specRefractWt,
                           float& clearcoatWt) {  // RT:537-550
  (void)eta;
  float r_diffuse = (1.0f - material.metallic) * (1.0f - material.transmission) * Luminance(material.baseColor);
  float r_specular = Luminance(mix(specCol, vec3(1.0f), approxFresnel));
  float r_clearcoat = (1.0f - material.metallic) * 0.25f * material.clearcoat;
  float r_refraction = (1.0f - material.metallic) * material.transmission * Luminance(material.baseColor) *
                       (1.0f - approxFresnel);
  float r_sum_inv = 1.0f / (r_diffuse + r_specular + r_clearcoat + r_refraction);
  diffuseWeight = r_diffuse * r_sum_inv;
  specReflectWt = r_specular * r_sum_inv;
  clearcoatWt = r_clearcoat * r_sum_inv;
  specRefractWt = r_refraction * r_sum_inv;
}

// RNG: Thomas Wang hash chained through the global wseed (RT:573-586)
float rand_(Ctx& C) {
  uint32_t seed = C.wseed;
  seed = (seed ^ 61u) ^ (seed >> 16u);
  seed *= 9u;
  seed = seed ^ (seed >> 4u);
  seed *= 0x27d4eb2du;
  C.wseed = seed ^ (seed >> 15u);
  return (float)C.wseed * (1.0f / 4294967296.0f);
}

// Sobol direction numbers RT:590-592 (8 dims x 32)
const uint32_t V[8 * 32] = {
2147483648u, 1073741824u, 536870912u, 268435456u, 134217728u, 67108864u, 33554432u, 16777216u, 8388608u, 4194304u, 2097152u, 1048576u, 524288u, 262144u, 131072u, 65536u, 32768u, 16384u, 8192u, 4096u, 2048u, 1024u, 512u, 256u, 128u, 64u, 32u, 16u, 8u, 4u, 2u, 1u,
2147483648u, 3221225472u, 2684354560u, 4026531840u, 2281701376u, 3422552064u, 2852126720u, 4278190080u, 2155872256u, 3233808384u, 2694840320u, 4042260480u, 2290614272u, 3435921408u, 2863267840u, 4294901760u, 2147516416u, 3221274624u, 2684395520u, 4026593280u, 2281736192u, 3422604288u, 2852170240u, 4278255360u, 2155905152u, 3233857728u, 2694881440u, 4042322160u, 2290649224u, 3435973836u, 2863311530u, 4294967295u,
2147483648u, 3221225472u, 1610612736u, 2415919104u, 3892314112u, 1543503872u, 2382364672u, 3305111552u, 1753219072u, 2629828608u, 3999268864u, 1435500544u, 2154299392u, 3231449088u, 1626210304u, 2421489664u, 3900735488u, 1556135936u, 2388680704u, 3314585600u, 1751705600u, 2627492864u, 4008611328u, 1431684352u, 2147543168u, 3221249216u, 1610649184u, 2415969680u, 3892340840u, 1543543964u, 2382425838u, 3305133397u,
2147483648u, 3221225472u, 536870912u, 1342177280u, 4160749568u, 1946157056u, 2717908992u, 2466250752u, 3632267264u, 624951296u, 1507852288u, 3872391168u, 2013790208u, 3020685312u, 2181169152u, 3271884800u, 546275328u, 1363623936u, 4226424832u, 1977167872u, 2693105664u, 2437829632u, 3689389568u, 635137280u, 1484783744u, 3846176960u, 2044723232u, 3067084880u, 2148008184u, 3222012020u, 537002146u, 1342505107u,
2147483648u, 1073741824u, 536870912u, 2952790016u, 4160749568u, 3690987520u, 2046820352u, 2634022912u, 1518338048u, 801112064u, 2707423232u, 4038066176u, 3666345984u, 1875116032u, 2170683392u, 1085997056u, 579305472u, 3016343552u, 4217741312u, 3719483392u, 2013407232u, 2617981952u, 1510979072u, 755882752u, 2726789248u, 4090085440u, 3680870432u, 1840435376u, 2147625208u, 1074478300u, 537900666u, 2953698205u,
2147483648u, 1073741824u, 1610612736u, 805306368u, 2818572288u, 335544320u, 2113929216u, 3472883712u, 2290089984u, 3829399552u, 3059744768u, 1127219200u, 3089629184u, 4199809024u, 3567124480u, 1891565568u, 394297344u, 3988799488u, 920674304u, 4193267712u, 2950604800u, 3977188352u, 3250028032u, 129093376u, 2231568512u, 2963678272u, 4281226848u, 432124720u, 803643432u, 1633613396u, 2672665246u, 3170194367u,
2147483648u, 3221225472u, 2684354560u, 3489660928u, 1476395008u, 2483027968u, 1040187392u, 3808428032u, 3196059648u, 599785472u, 505413632u, 4077912064u, 1182269440u, 1736704000u, 2017853440u, 2221342720u, 3329785856u, 2810494976u, 3628507136u, 1416089600u, 2658719744u, 864310272u, 3863387648u, 3076993792u, 553150080u, 272922560u, 4167467040u, 1148698640u, 1719673080u, 2009075780u, 2149644390u, 3222291575u,
2147483648u, 1073741824u, 2684354560u, 1342177280u, 2281701376u, 1946157056u, 436207616u, 2566914048u, 2625634304u, 3208642560u, 2720006144u, 2098200576u, 111673344u, 2354315264u, 3464626176u, 4027383808u, 2886631424u, 3770826752u, 1691164672u, 3357462528u, 1993345024u, 3752330240u, 873073152u, 2870150400u, 1700563072u, 87021376u, 1097028000u, 1222351248u, 1560027592u, 2977959924u, 23268898u, 437609937u};

int grayCode(int i) { return i ^ (i >> 1); }  // RT:598-600

float sobol(int d, int i) {  // RT:604-612; R8: V[] reads past 256 entries yield 0
  uint32_t result = 0u;
  int offset = d * 32;
  for (int j = 0; i != 0; i >>= 1, j++)
    if ((i & 1) != 0) {
      int k = j + offset;
      result ^= (k >= 0 && k < 256) ? V[k] : 0u;
    }
  return (float)result * (1.0f / (float)0xFFFFFFFFu);
}
vec2 sobolVec2(int i, int b) {  // RT:616-620
  float u = sobol(b * 2, grayCode(i));
  float v = sobol(b * 2 + 1, grayCode(i));
  return vec2{u, v};
}

vec2 toSphericalCoord(const Ctx& C, vec3 v) {  // RT:625-631 (R13: envAngle not wrapped)
  vec2 uv = vec2{atan2_(v.z, v.x), asin_(v.y)};
  uv.x = uv.x / (2.0f * PI);
  uv.y = uv.y / PI;
  uv.x = uv.x + 0.5f;
  uv.y = uv.y + 0.5f;
  uv.y = 1.0f - uv.y;
  return vec2{uv.x + C.f->env_angle, uv.y + 0.0f};
}

vec3 SampleHdr(Ctx& C, float xi_1, float xi_2) {  // RT:635-646 (R13: s = xi_1)
  C.c.cache_fetches++;
  vec3 c = tex2D(C.s->hdr_cache, C.s->hdr_w, C.s->hdr_h, vec2{xi_1, xi_2});
  vec2 xy = vec2{c.x, c.y};
  xy.y = 1.0f - xy.y;
  float phi = 2.0f * PI * (xy.x - 0.5f);
  float theta = PI * (xy.y - 0.5f);
  return vec3(cos_(theta) * cos_(phi), sin_(theta), cos_(theta) * sin_(phi));
}

vec3 CosineSampleHemisphere(float r1, float r2) {  // RT:650-659
  vec3 dir;
  float r = sqrt_(r1);
  float phi = TWO_PI * r2;
  dir.x = r * cos_(phi);
  dir.y = r * sin_(phi);
  dir.z = sqrt_(max_(0.0f, 1.0f - dir.x * dir.x - dir.y * dir.y));
  return dir;
}

vec3 SampleGTR1(float rgh, float r1, float r2) {  // RT:716-729 (R23: r1 used twice)
  (void)r2;
  float a = max_(0.001f, rgh);
  float a2 = a * a;
  float phi = r1 * TWO_PI;
  float cosTheta = sqrt_((1.0f - pow_(a2, 1.0f - r1)) / (1.0f - a2));
  float sinTheta = clamp_(sqrt_(1.0f - (cosTheta * cosTheta)), 0.0f, 1.0f);
  float sinPhi = sin_(phi);
  float cosPhi = cos_(phi);
  return vec3(sinTheta * cosPhi, sinTheta * sinPhi, cosTheta);
}

vec3 SampleGGXVNDF(vec3 V_, float ax, float ay, float r1, float r2) {  // RT:751-769
  vec3 Vh = normalize(vec3(ax * V_.x, ay * V_.y, V_.z));
  float lensq = Vh.x * Vh.x + Vh.y * Vh.y;
  vec3 T1 = lensq > 0 ? vec3(-Vh.y, Vh.x, 0) * inversesqrt_(lensq) : vec3(1, 0, 0);
  vec3 T2 = cross(Vh, T1);
  float r = sqrt_(r1);
  float phi = 2.0f * PI * r2;
  float t1 = r * cos_(phi);
  float t2 = r * sin_(phi);
  float s = 0.5f * (1.0f + Vh.z);
  t2 = (1.0f - s) * sqrt_(1.0f - t1 * t1) + s * t2;
  vec3 Nh = t1 * T1 + t2 * T2 + sqrt_(max_(0.0f, 1.0f - t1 * t1 - t2 * t2)) * Vh;
  return normalize(vec3(ax * Nh.x, ay * Nh.y, max_(0.0f, Nh.z)));
}

vec2 CranleyPattersonRotation(Ctx& C, vec2 p) {  // RT:772-785
  float u = rand_(C);
  float v = rand_(C);
  p.x += u;
  if (p.x > 1) p.x -= 1;
  if (p.x < 0) p.x += 1;
  p.y += v;
  if (p.y > 1) p.y -= 1;
  if (p.y < 0) p.y += 1;
  return p;
}

vec3 EvalDiffuse(const Material& mat, vec3 Csheen, vec3 V_, vec3 L, vec3 H, float& pdf) {  // RT:925-948
  pdf = 0.0f;
  if (L.z <= 0.0f) return vec3(0.0f);
  float FL = SchlickFresnel(L.z);
  float FV = SchlickFresnel(V_.z);
  float FH = SchlickFresnel(dot(L, H));
  float Fd90 = 0.5f + 2.0f * dot(L, H) * dot(L, H) * mat.roughness;
  float Fd = mix_(1.0f, Fd90, FL) * mix_(1.0f, Fd90, FV);
  float Fss90 = dot(L, H) * dot(L, H) * mat.roughness;
  float Fss = mix_(1.0f, Fss90, FL) * mix_(1.0f, Fss90, FV);
  float ss = 1.25f * (Fss * (1.0f / (L.z + V_.z) - 0.5f) + 0.5f);
  vec3 Fsheen = FH * mat.sheen * Csheen;
  pdf = L.z * INV_PI;
  return (1.0f - mat.metallic) * (1.0f - mat.transmission) *
         (INV_PI * mix_(Fd, ss, mat.subsurface) * mat.baseColor + Fsheen);
}

vec3 EvalSpecReflection(const Material& mat, float eta, vec3 specCol, vec3 V_, vec3 L, vec3 H,
                        float& pdf) {  // RT:950-964
  pdf = 0.0f;
  if (L.z <= 0.0f) return vec3(0.0f);
  float FM = DisneyFresnel(mat, eta, dot(L, H), dot(V_, H));
  vec3 F = mix(specCol, vec3(1.0f), FM);
  float D = GTR2_Aniso(H.z, H.x, H.y, mat.ax, mat.ay);
  float G1 = SmithG_GGX_Aniso(fabs_(V_.z), V_.x, V_.y, mat.ax, mat.ay);
  float G2 = G1 * SmithG_GGX_Aniso(fabs_(L.z), L.x, L.y, mat.ax, mat.ay);
  pdf = G1 * D / (4.0f * V_.z);
  return F * D * G2 / (4.0f * L.z * V_.z);
}

vec3 EvalSpecRefraction(const Material& mat, float eta, vec3 V_, vec3 L, vec3 H, float& pdf) {  // RT:966-984
  pdf = 0.0f;
  if (L.z >= 0.0f) return vec3(1.0f, 0.0f, 0.0f);  // R26
  float F = DielectricFresnel(fabs_(dot(V_, H)), eta);
  float D = GTR2_Aniso(H.z, H.x, H.y, mat.ax, mat.ay);
  float G1 = SmithG_GGX_Aniso(fabs_(V_.z), V_.x, V_.y, mat.ax, mat.ay);
  float G2 = G1 * SmithG_GGX_Aniso(fabs_(L.z), L.x, L.y, mat.ax, mat.ay);
  float denom = dot(L, H) + dot(V_, H) * eta;
  denom *= denom;
  float eta2 = eta * eta;
  float jacobian = fabs_(dot(L, H)) / denom;
  pdf = G1 * max_(0.0f, dot(V_, H)) * D * jacobian / V_.z;
  return pow3(mat.baseColor, vec3(0.5f)) * (1.0f - mat.metallic) * mat.transmission * (1.0f - F) * D * G2 *
         fabs_(dot(V_, H)) * jacobian * eta2 / fabs_(L.z * V_.z);
}

vec3 EvalClearcoat(const Material& mat, vec3 V_, vec3 L, vec3 H, float& pdf) {  // RT:986-1000 (R23)
  pdf = 0.0f;
  if (L.z <= 0.0f) return vec3(0.0f);
  float FH = DielectricFresnel(dot(V_, H), 1.0f / 1.5f);
  float F = mix_(0.04f, 1.0f, FH);
  float D = GTR1(H.z, mat.clearcoatGloss);
  float G = SmithG_GGX(L.z, 0.25f) * SmithG_GGX(V_.z, 0.25f);
  float jacobian = 1.0f / (4.0f * dot(V_, H));
  pdf = D * H.z * jacobian;
  return vec3(0.25f) * mat.clearcoat * F * D * G / (4.0f * L.z * V_.z);
}

vec3 DisneyEval(const Material& material, vec3 V_, vec3 N, vec3 L, float& bsdfPdf) {  // RT:1002-1067
  bsdfPdf = 0.0f;
  vec3 f = vec3(0.0f);
  float eta = dot(V_, N) > 0.0f ? (1.0f / material.IOR) : material.IOR;  // R10
  vec3 T, B;
  getTangent(N, T, B);
  V_ = ToLocal(T, B, N, V_);
  L = ToLocal(T, B, N, L);
  vec3 H;
  if (L.z > 0.0f) H = normalize(L + V_);
  else H = normalize(L + V_ * eta);
  if (H.z < 0.0f) H = -H;
  vec3 specCol, sheenCol;
  GetSpecColor(material, eta, specCol, sheenCol);
  float diffuseWt, specReflectWt, specRefractWt, clearcoatWt;
  float fresnel = DisneyFresnel(material, eta, dot(L, H), dot(V_, H));
  CalculateBSDFLobePdfs(material, eta, specCol, fresnel, diffuseWt, specReflectWt, specRefractWt, clearcoatWt);
  float pdf;
  if (diffuseWt > 0.0f && L.z > 0.0f) {
    f = f + EvalDiffuse(material, sheenCol, V_, L, H, pdf);
    bsdfPdf += pdf * diffuseWt;
  }
  if (specReflectWt > 0.0f && L.z > 0.0f && V_.z > 0.0f) {
    f = f + EvalSpecReflection(material, eta, specCol, V_, L, H, pdf);
    bsdfPdf += pdf * specReflectWt;
  }
  if (specRefractWt > 0.0f && L.z < 0.0f) {
    f = f + EvalSpecRefraction(material, eta, V_, L, H, pdf);
    bsdfPdf += pdf * specRefractWt;
  }
  if (clearcoatWt > 0.0f && L.z > 0.0f && V_.z > 0.0f) {
    f = f + EvalClearcoat(material, V_, L, H, pdf);
    bsdfPdf += pdf * clearcoatWt;
  }
  return f * fabs_(L.z);
}

vec3 DisneySample(float xi_1, float xi_2, float xi_3, const Material& material, vec3 V_, vec3 N, vec3& L,
                  float& pdf, bool& isRefract) {  // RT:1070-1161
  pdf = 0.0f;
  vec3 f = vec3(0.0f);
  isRefract = false;
  float r1 = xi_1;
  float r2 = xi_2;
  float eta = dot(V_, N) > 0.0f ? (1.0f / material.IOR) : material.IOR;
  vec3 T, B;
  getTangent(N, T, B);
  V_ = ToLocal(T, B, N, V_);
  vec3 specCol, sheenCol;
  GetSpecColor(material, eta, specCol, sheenCol);
  float diffuseWt, specReflectWt, specRefractWt, clearcoatWt;
  float approxFresnel = DisneyFresnel(material, eta, V_.z, V_.z);
  CalculateBSDFLobePdfs(material, eta, specCol, approxFresnel, diffuseWt, specReflectWt, specRefractWt, clearcoatWt);
  float cdf[4];
  cdf[0] = diffuseWt;
  cdf[1] = cdf[0] + clearcoatWt;
  cdf[2] = cdf[1] + specReflectWt;
  cdf[3] = cdf[2] + specRefractWt;
  L = vec3(0.0f);  // R7: GLSL leaves the out-param undefined until written; restated as 0
  if (r1 < cdf[0]) {
    r1 /= cdf[0];
    L = CosineSampleHemisphere(r1, r2);
    vec3 H = normalize(L + V_);
    f = EvalDiffuse(material, sheenCol, V_, L, H, pdf);
    pdf *= diffuseWt;
  } else if (r1 < cdf[1]) {
    r1 = (r1 - cdf[0]) / (cdf[1] - cdf[0]);
    vec3 H = SampleGTR1(material.clearcoatGloss, r1, r2);
    if (H.z < 0.0f) H = -H;
    L = normalize(reflect(-V_, H));
    f = EvalClearcoat(material, V_, L, H, pdf);
    pdf *= clearcoatWt;
  } else {
    r1 = (r1 - cdf[1]) / (1.0f - cdf[1]);
    vec3 H = SampleGGXVNDF(V_, material.ax, material.ay, r1, r2);
    if (H.z < 0.0f) H = -H;
    float fresnel = DisneyFresnel(material, eta, dot(L, H), dot(V_, H));  // R7: L == 0 here
    float F = 1.0f - ((1.0f - fresnel) * material.transmission * (1.0f - material.metallic));
    if (xi_3 < F) {
      L = normalize(reflect(-V_, H));
      f = EvalSpecReflection(material, eta, specCol, V_, L, H, pdf);
      pdf *= F;
    } else {
      isRefract = true;
      L = normalize(refract(-V_, H, eta));  // R14: TIR -> refract = 0 -> NaN
      f = EvalSpecRefraction(material, eta, V_, L, H, pdf);
      pdf *= (1.0f - F);
    }
    pdf *= specReflectWt + specRefractWt;
  }
  L = ToWorld(T, B, N, L);
  return f * fabs_(dot(N, L));
}

vec3 hdrColor(Ctx& C, vec3 L) {  // RT:1165-1169
  C.c.env_fetches++;
  vec2 uv = toSphericalCoord(C, normalize(L));
  return tex2D(C.s->hdr_map, C.s->hdr_w, C.s->hdr_h, uv);
}

float hdrPdf(Ctx& C, vec3 L, int hdrResolution) {  // RT:1173-1186
  C.c.cache_fetches++;
  vec2 uv = toSphericalCoord(C, normalize(L));
  float pdf = tex2D(C.s->hdr_cache, C.s->hdr_w, C.s->hdr_h, uv).z;
  float theta = PI * uv.y;
  float sin_theta = max_(sin_(theta), 1e-10f);
  float p_convert = (float)(hdrResolution * hdrResolution / 2) / (TWO_PI * PI * sin_theta);
  return pdf * p_convert;
}

vec3 getDefaultSkyColor(float y) {  // RT:1190-1193
  float t = 0.5f * (y + 1.0f);
  return (1.0f - t) * vec3(1.0f, 1.0f, 1.0f) + t * vec3(0.5f, 0.7f, 1.0f);
}

vec3 SampleHG(vec3 V_, float g, float r1, float r2) {  // RT:1195-1216
  float cosTheta;
  if (fabs_(g) < 0.001f) cosTheta = 1 - 2 * r2;
  else {
    float sqrTerm = (1 - g * g) / (1 + g - 2 * g * r2);
    cosTheta = -(1 + g * g - sqrTerm * sqrTerm) / (2 * g);
  }
  float phi = r1 * TWO_PI;
  float sinTheta = clamp_(sqrt_(1.0f - (cosTheta * cosTheta)), 0.0f, 1.0f);
  float sinPhi = sin_(phi);
  float cosPhi = cos_(phi);
  vec3 v1, v2;
  getTangent(V_, v1, v2);
  return sinTheta * cosPhi * v1 + sinTheta * sinPhi * v2 + cosTheta * V_;
}

float PhaseHG(float cosTheta, float g) {  // RT:1218-1222
  float denom = 1 + g * g + 2 * g * cosTheta;
  return INV_4_PI * (1 - g * g) / (denom * sqrt_(denom));
}

float misMixWeight(float a, float b) {  // RT:1285-1288
  float t = a * a;
  return t / (b * b + t);
}

vec3 shadingImportanceSampling_BSDF(Ctx& C, HitRecord hit) {  // RT:1369-1516
  const orc_frame* F = C.f;
  vec3 Lo = vec3(0);
  vec3 history = vec3(1);
  for (int i = 0; i < F->max_bounce; i++) {
    vec3 V_ = -hit.viewDir;
    vec3 N = hit.normal;
    Ray hdrTestRay;
    hdrTestRay.origin = hit.hitPoint;
    float xa = rand_(C);  // R24: GLSL evaluates SampleHdr(rand(), rand()) left to right
    float xb = rand_(C);
    hdrTestRay.direction = SampleHdr(C, xa, xb);
    if (dot(N, hdrTestRay.direction) > 0.0f) {
      HitRecord hdrHit = hitBVH(C, hdrTestRay);
      if (!hdrHit.isHit) {
        vec3 L = hdrTestRay.direction;
        float light_pdf = hdrPdf(C, L, C.s->hdr_resolution);
        vec3 light_fr = hdrColor(C, L) * F->env_intensity;
        float disney_eval_pdf;
        vec3 disney_eval_fr = DisneyEval(hit.material, V_, N, L, disney_eval_pdf);
        float mis_weight = misMixWeight(light_pdf, disney_eval_pdf);
        if (!F->enable_mis) mis_weight = 1.0f;
        Lo = Lo + mis_weight * history * light_fr * disney_eval_fr / light_pdf;
      }
    }
    vec2 uv = sobolVec2(C.f->loop_num + 1, i);
    uv = CranleyPattersonRotation(C, uv);
    float xi_1 = uv.x;
    float xi_2 = uv.y;
    float xi_3 = rand_(C);
    float disney_sample_pdf = 0.0f;
    vec3 disney_sample_fr = vec3(0);
    vec3 L = vec3(0);
    bool isRefract;
    disney_sample_fr = DisneySample(xi_1, xi_2, xi_3, hit.material, V_, N, L, disney_sample_pdf, isRefract);
    bool mediumSampled = false;
    float scatter_pdf = 0.0f;
    float transmittance = 1.0f;
    if (disney_sample_pdf > 0.0f) {
      if (!isRefract) {
        history = history * (disney_sample_fr / disney_sample_pdf);
      } else {
        // R9: refraction skips f/pdf; R11: absorption over the pre-hit segment
        if (hit.material.medium.type == MEDIUM_ABSORB) {
          history = history * exp3(-(vec3(1.0f) - hit.material.medium.color) * hit.distance *
                                   hit.material.medium.density);
        } else if (hit.material.medium.type == MEDIUM_EMISSIVE) {
          Lo = Lo + hit.material.medium.color * hit.distance * hit.material.medium.density * history;
        } else if (hit.material.medium.type == MEDIUM_SCATTER) {
          float scatterDist = min_(-log_(xi_3) / hit.material.medium.density, hit.distance);
          mediumSampled = scatterDist < hit.distance;
          if (mediumSampled) {
            transmittance *= exp_(-1.0f * scatterDist);
            history = history * (hit.material.medium.color * transmittance);
            hit.hitPoint = hit.hitPoint + hit.viewDir * scatterDist;
            vec3 scatterDir = SampleHG(V_, hit.material.medium.anisotropy, xi_1, xi_2);
            scatter_pdf = PhaseHG(dot(V_, scatterDir), hit.material.medium.anisotropy);
            L = scatterDir;
          }
        }
      }
    } else {
      break;
    }
    float disney_eval_pdf = 0.0f;
    vec3 disney_eval_fr = vec3(0);
    disney_eval_fr = DisneyEval(hit.material, V_, N, L, disney_eval_pdf);
    if (mediumSampled && scatter_pdf > 0.0f) {
      disney_eval_pdf = scatter_pdf;
      disney_eval_fr = vec3(scatter_pdf);
    }
    Ray randomRay;
    randomRay.origin = hit.hitPoint;
    randomRay.direction = L;
    HitRecord nextHit = hitBVH(C, randomRay);
    if (!nextHit.isHit) {
      vec3 light_fr = vec3(0);
      if (F->enable_env_map) {
        light_fr = hdrColor(C, L) * F->env_intensity;
        float light_pdf = hdrPdf(C, L, C.s->hdr_resolution);
        float mis_weight = misMixWeight(disney_eval_pdf, light_pdf);
        if (!F->enable_mis) mis_weight = 1.0f;
        if (!mediumSampled) Lo = Lo + mis_weight * history * light_fr * disney_eval_fr / disney_eval_pdf;  // R9, R14
        else Lo = Lo + history * light_fr * disney_eval_fr / light_pdf;
      } else {
        light_fr = getDefaultSkyColor(randomRay.direction.y);
        Lo = Lo + history * light_fr * disney_eval_fr / disney_eval_pdf;
      }
      break;
    }
    vec3 Le = nextHit.material.emissive;
    Lo = Lo + history * Le * disney_eval_fr / disney_eval_pdf;
    hit = nextHit;
  }
  return Lo;
}

// ---------------------------------------------------------------- BRDF mode RT:520-921, 1290-1367
void CalculateBRDFLobePdfs(const Material& material, float& pDiffuse, float& pSpecular, float& pClearcoat) {  // RT:520-533
  float r_diffuse = (1.0f - material.metallic);
  float r_specular = (1.0f - material.metallic) + material.metallic;
  float r_clearcoat = (1.0f - material.metallic) * 0.25f * material.clearcoat;
  float r_sum_inv = 1.0f / (r_diffuse + r_specular + r_clearcoat);
  pDiffuse = r_diffuse * r_sum_inv;
  pSpecular = r_specular * r_sum_inv;
  pClearcoat = r_clearcoat * r_sum_inv;
}
vec3 toNormalHemisphere(vec3 v, vec3 N) {  // RT:663-669
  vec3 helper = vec3(1, 0, 0);
  if (fabs_(N.x) > 0.999f) helper = vec3(0, 0, 1);
  vec3 tangent = normalize(cross(N, helper));
  vec3 bitangent = normalize(cross(N, tangent));
  return v.x * tangent + v.y * bitangent + v.z * N;
}
vec3 SampleCosineHemisphere(float xi_1, float xi_2, vec3 N) {  // RT:673-685
  float r = sqrt_(xi_1);
  float theta = xi_2 * TWO_PI;
  float x = r * cos_(theta);
  float y = r * sin_(theta);
  float z = sqrt_(1.0f - x * x - y * y);
  return toNormalHemisphere(vec3(x, y, z), N);
}
vec3 SampleGTR1_h(float xi_1, float xi_2, vec3 V_, vec3 N, float alpha) {  // RT:697-714
  float phi_h = xi_1 * TWO_PI;
  float sin_phi_h = sin_(phi_h);
  float cos_phi_h = cos_(phi_h);
  float cos_theta_h = sqrt_((1.0f - pow_(alpha * alpha, 1.0f - xi_2)) / (1.0f - alpha * alpha));
  float sin_theta_h = sqrt_(max_(0.0f, 1.0f - cos_theta_h * cos_theta_h));
  vec3 H = vec3(sin_theta_h * cos_phi_h, sin_theta_h * sin_phi_h, cos_theta_h);
  H = toNormalHemisphere(H, N);
  return reflect(-V_, H);
}
vec3 SampleGTR2(float xi_1, float xi_2, vec3 V_, vec3 N, float alpha) {  // RT:732-749
  float phi_h = 2.0f * PI * xi_1;
  float sin_phi_h = sin_(phi_h);
  float cos_phi_h = cos_(phi_h);
  float cos_theta_h = sqrt_((1.0f - xi_2) / (1.0f + (alpha * alpha - 1.0f) * xi_2));
  float sin_theta_h = sqrt_(max_(0.0f, 1.0f - cos_theta_h * cos_theta_h));
  vec3 H = vec3(sin_theta_h * cos_phi_h, sin_theta_h * sin_phi_h, cos_theta_h);
  H = toNormalHemisphere(H, N);
  return reflect(-V_, H);
}
vec3 SampleBRDF(float xi_1, float xi_2, float xi_3, vec3 V_, vec3 N, const Material& material) {  // RT:789-833
  float p_diffuse, p_specular, p_clearcoat;
  CalculateBRDFLobePdfs(material, p_diffuse, p_specular, p_clearcoat);
  float alpha_GTR1 = mix_(0.1f, 0.001f, material.clearcoatGloss);
  float alpha_GTR2 = max_(0.001f, sqr(material.roughness));
  float cdf[3];
  cdf[0] = p_diffuse;
  cdf[1] = cdf[0] + p_clearcoat;
  cdf[2] = cdf[1] + p_specular;
  float rd = xi_3;
  // RT:808-817 compute eta, a VNDF half vector and a Fresnel that are never used
  if (rd <= cdf[0]) return SampleCosineHemisphere(xi_1, xi_2, N);
  else if (rd <= cdf[1]) return SampleGTR1_h(xi_1, xi_2, V_, N, alpha_GTR1);
  else if (rd <= cdf[2]) return SampleGTR2(xi_1, xi_2, V_, N, alpha_GTR2);
  return vec3(0, 1, 0);
}
vec3 BRDF_Evaluate(vec3 V_, vec3 N, vec3 L, vec3 X, vec3 Y, const Material& material, float& pdf) {  // RT:836-921
  pdf = 1e-10f;
  float NdotL = dot(N, L);
  float NdotV = dot(N, V_);
  if (NdotL < 0 || NdotV < 0) return vec3(0);
  vec3 H = normalize(L + V_);
  float NdotH = dot(N, H);
  float LdotH = dot(L, H);
  float VdotH = dot(V_, H);
  (void)VdotH;
  vec3 Cdlin = material.baseColor;
  float Cdlum = Luminance(Cdlin);
  vec3 Ctint = (Cdlum > 0) ? (Cdlin / Cdlum) : vec3(1);
  vec3 Cspec = material.specular * mix(vec3(1), Ctint, material.specularTint);
  vec3 Cspec0 = mix(0.08f * Cspec, Cdlin, material.metallic);
  vec3 Csheen = mix(vec3(1), Ctint, material.sheenTint);
  float Fd90 = 0.5f + 2.0f * LdotH * LdotH * material.roughness;
  float FL = SchlickFresnel(NdotL);
  float FV = SchlickFresnel(NdotV);
  float Fd = mix_(1.0f, Fd90, FL) * mix_(1.0f, Fd90, FV);
  float Fss90 = LdotH * LdotH * material.roughness;
  float Fss = mix_(1.0f, Fss90, FL) * mix_(1.0f, Fss90, FV);
  float ss = 1.25f * (Fss * (1.0f / (NdotL + NdotV) - 0.5f) + 0.5f);
  float FH = SchlickFresnel(LdotH);
  float alpha = max_(0.001f, sqr(material.roughness));
  float Ds = GTR2(NdotH, alpha);
  vec3 Fs = mix(Cspec0, vec3(1), FH);
  float Gs = SmithG_GGX(NdotL, material.roughness);  // R27: roughness, not alpha
  Gs *= SmithG_GGX(NdotV, material.roughness);
  if (material.anisotropic > 0) {
    Ds = GTR2_Aniso(NdotH, dot(H, X), dot(H, Y), material.ax, material.ay);
    Gs = SmithG_GGX_Aniso(NdotL, dot(L, X), dot(L, Y), material.ax, material.ay);
    Gs *= SmithG_GGX_Aniso(NdotV, dot(V_, X), dot(V_, Y), material.ax, material.ay);
  }
  float Dr = GTR1(NdotH, mix_(0.1f, 0.001f, 1.0f - material.clearcoatGloss));
  float Fr = mix_(0.04f, 1.0f, FH);
  float Gr = SmithG_GGX(NdotL, 0.25f) * SmithG_GGX(NdotV, 0.25f);
  vec3 Fsheen = FH * material.sheen * Csheen;
  vec3 diffuse = INV_PI * mix_(Fd, ss, material.subsurface) * Cdlin + Fsheen;
  vec3 specular = Gs * Fs * Ds / (4.0f * NdotV * NdotL);
  vec3 clearcoat = vec3(0.25f) * Gr * Fr * Dr * material.clearcoat / (4.0f * NdotV * NdotL);
  float p_diffuse, p_specular, p_clearcoat;
  CalculateBRDFLobePdfs(material, p_diffuse, p_specular, p_clearcoat);
  float pdf_diffuse = NdotL * INV_PI;
  float pdf_specular = Ds * NdotH / (4.0f * LdotH);
  float pdf_clearcoat = Dr * NdotH / (4.0f * LdotH);
  pdf = p_diffuse * pdf_diffuse + p_specular * pdf_specular + p_clearcoat * pdf_clearcoat;
  pdf = max_(1e-10f, pdf);
  return (1.0f - material.metallic) * diffuse + specular + clearcoat;
}

vec3 shadingImportanceSampling_BRDF(Ctx& C, HitRecord hit) {  // RT:1290-1367
  const orc_frame* F = C.f;
  vec3 Lo = vec3(0);
  vec3 history = vec3(1);
  for (int i = 0; i < F->max_bounce; i++) {
    vec3 V_ = -hit.viewDir;
    vec3 N = hit.normal;
    Ray hdrTestRay;
    hdrTestRay.origin = hit.hitPoint;
    float xa = rand_(C);
    float xb = rand_(C);
    hdrTestRay.direction = SampleHdr(C, xa, xb);
    vec3 tangent, bitangent;
    getTangent(N, tangent, bitangent);
    if (dot(N, hdrTestRay.direction) > 0.0f) {
      HitRecord hdrHit = hitBVH(C, hdrTestRay);
      if (!hdrHit.isHit) {
        vec3 L = hdrTestRay.direction;
        float light_pdf = hdrPdf(C, L, C.s->hdr_resolution);
        vec3 light_fr = hdrColor(C, L) * F->env_intensity;
        float disney_brdf_pdf;
        vec3 disney_brdf_fr = BRDF_Evaluate(V_, N, L, tangent, bitangent, hit.material, disney_brdf_pdf);
        float mis_weight = misMixWeight(light_pdf, disney_brdf_pdf);
        Lo = Lo + mis_weight * history * light_fr * disney_brdf_fr * fabs_(dot(N, L)) / light_pdf;
      }
    }
    vec2 uv = sobolVec2(C.f->loop_num + 1, i);
    uv = CranleyPattersonRotation(C, uv);
    float xi_1 = uv.x, xi_2 = uv.y;
    float xi_3 = rand_(C);
    vec3 L = SampleBRDF(xi_1, xi_2, xi_3, V_, N, hit.material);
    float NdotL = dot(N, L);
    float pdf_brdf;
    vec3 f_r = BRDF_Evaluate(V_, N, L, tangent, bitangent, hit.material, pdf_brdf);
    if (pdf_brdf <= 0.0f) break;
    history = history * (f_r * fabs_(NdotL) / pdf_brdf);
    Ray randomRay;
    randomRay.origin = hit.hitPoint;
    randomRay.direction = L;
    HitRecord newHit = hitBVH(C, randomRay);
    if (!newHit.isHit) {
      vec3 skyColor = vec3(0);
      if (F->enable_env_map) {
        skyColor = hdrColor(C, L) * F->env_intensity;
        float pdf_light = hdrPdf(C, L, C.s->hdr_resolution);
        float mis_weight = misMixWeight(pdf_brdf, pdf_light);
        Lo = Lo + mis_weight * history * skyColor * f_r * fabs_(NdotL) / pdf_brdf;
      } else {
        skyColor = getDefaultSkyColor(randomRay.direction.y);
        Lo = Lo + history * skyColor * f_r * fabs_(NdotL) / pdf_brdf;
      }
      break;
    }
    vec3 Le = newHit.material.emissive;
    Lo = Lo + history * Le * f_r * fabs_(NdotL) / pdf_brdf;
    hit = newHit;
  }
  return Lo;
}

// ----------------------------------------------------------------------- main RT:1518-1558
vec3 shade_pixel(Ctx& C, float u, float v, vec3 hist) {
  const orc_frame* F = C.f;
  C.wseed = (uint32_t)(C.f->rand_origin * 6.95857f * (u * v));  // R5
  if (F->max_iterations == -1 || F->loop_num < F->max_iterations) {  // R12
    C.c.samples++;
    Ray cameraRay;
    cameraRay.origin = vec3(F->position[0], F->position[1], F->position[2]);
    vec3 lbc = vec3(F->left_bottom_corner[0], F->left_bottom_corner[1], F->left_bottom_corner[2]);
    vec3 right = vec3(F->right[0], F->right[1], F->right[2]);
    vec3 up = vec3(F->up[0], F->up[1], F->up[2]);
    cameraRay.direction = normalize(lbc + (u * 2.0f * F->half_w) * right + (v * 2.0f * F->half_h) * up);  // R6
    HitRecord firstHit = hitBVH(C, cameraRay);
    vec3 curColor = vec3(1);
    if (!firstHit.isHit) {
      if (F->enable_env_map) curColor = hdrColor(C, cameraRay.direction) * F->env_intensity;
      else curColor = getDefaultSkyColor(cameraRay.direction.y);
    } else {
      vec3 Le = firstHit.material.emissive;
      vec3 Li = vec3(0);
      if (F->enable_bsdf) Li = shadingImportanceSampling_BSDF(C, firstHit);
      else Li = shadingImportanceSampling_BRDF(C, firstHit);
      curColor = Le + Li;
    }
    // RT:1552 (R14: NaN history stays NaN through 0*NaN)
    curColor = (1.0f / (float)F->loop_num) * curColor +
               ((float)(F->loop_num - 1) / (float)F->loop_num) * hist;
    return curColor;
  }
  return hist;
}

}  // namespace

extern "C" {

// Render n_frames progressive frames over the sub-rectangle [x0,x0+w) x [y0,y0+h) of a
// W x H frame.  accum (w*h*3 floats, row-major over the sub-rect) is the history
// texture on entry and the new accumulation on exit.  Frame k uses frames[k].
int orc_render(const orc_scene* scene, const orc_frame* frames, int n_frames, int W, int H, int x0, int y0,
               int w, int h, float* accum, orc_counters* counters, int n_threads) {
  if (!scene || !frames || !accum || W <= 0 || H <= 0 || w < 0 || h < 0) return -1;
  if (x0 < 0 || y0 < 0 || x0 + w > W || y0 + h > H) return -2;
  orc_counters total;
  memset(&total, 0, sizeof(total));
#ifdef _OPENMP
  if (n_threads > 0) omp_set_num_threads(n_threads);
#else
  (void)n_threads;
#endif
  long npix = (long)w * h;
#pragma omp parallel
  {
    orc_counters local;
    memset(&local, 0, sizeof(local));
#pragma omp for schedule(dynamic, 64)
    for (long p = 0; p < npix; p++) {
      int px = x0 + (int)(p % w);
      int py = y0 + (int)(p / w);
      // TexCoords of the full-screen quad at the fragment centre (vertex_shader.glsl)
      float u = ((float)px + 0.5f) / (float)W;
      float v = ((float)py + 0.5f) / (float)H;
      float* a = accum + 3 * p;
      vec3 hist = vec3(a[0], a[1], a[2]);
      for (int k = 0; k < n_frames; k++) {
        Ctx C;
        C.s = scene; C.f = &frames[k]; C.wseed = 0;
        memset(&C.c, 0, sizeof(C.c));
        hist = shade_pixel(C, u, v, hist);
        local.rays += C.c.rays; local.internal_pops += C.c.internal_pops;
        local.leaf_pops += C.c.leaf_pops; local.tri_tests += C.c.tri_tests;
        local.closer_updates += C.c.closer_updates; local.samples += C.c.samples;
        local.env_fetches += C.c.env_fetches; local.cache_fetches += C.c.cache_fetches;
      }
      a[0] = hist.x; a[1] = hist.y; a[2] = hist.z;
    }
#pragma omp critical
    {
      total.rays += local.rays; total.internal_pops += local.internal_pops;
      total.leaf_pops += local.leaf_pops; total.tri_tests += local.tri_tests;
      total.closer_updates += local.closer_updates; total.samples += local.samples;
      total.env_fetches += local.env_fetches; total.cache_fetches += local.cache_fetches;
    }
  }
  if (counters) *counters = total;
  return 0;
}

// Single-ray closest-hit query (known-answer tests of RT:338-392).
int orc_trace(const orc_scene* scene, const float* origin, const float* dir, float* out_distance,
              float* out_point, float* out_normal, int* out_inside) {
  orc_frame f;
  memset(&f, 0, sizeof(f));
  Ctx C;
  C.s = scene; C.f = &f; C.wseed = 0;
  memset(&C.c, 0, sizeof(C.c));
  Ray r;
  r.origin = vec3(origin[0], origin[1], origin[2]);
  r.direction = vec3(dir[0], dir[1], dir[2]);
  HitRecord h = hitBVH(C, r);
  *out_distance = h.isHit ? h.distance : -1.0f;
  if (h.isHit) {
    out_point[0] = h.hitPoint.x; out_point[1] = h.hitPoint.y; out_point[2] = h.hitPoint.z;
    out_normal[0] = h.normal.x; out_normal[1] = h.normal.y; out_normal[2] = h.normal.z;
    *out_inside = h.isInside ? 1 : 0;
  }
  return h.isHit ? 1 : 0;
}

// Builtin/RNG probes for known-answer tests.
float orc_wang_rand(uint32_t* seed) {
  Ctx C; C.wseed = *seed;
  float r = rand_(C);
  *seed = C.wseed;
  return r;
}
float orc_sobol(int d, int i) { return sobol(d, i); }
void orc_sobol_vec2(int i, int b, float* out) { vec2 v = sobolVec2(i, b); out[0] = v.x; out[1] = v.y; }
float orc_math(int fn, float x, float y) {
  switch (fn) {
    case 0: return sin_(x);
    case 1: return cos_(x);
    case 2: return atan2_(x, y);
    case 3: return asin_(x);
    case 4: return exp_(x);
    case 5: return log_(x);
    case 6: return pow_(x, y);
    default: return 0.0f;
  }
}
float orc_dielectric_fresnel(float cos_i, float eta) { return DielectricFresnel(cos_i, eta); }
float orc_gtr2(float ndoth, float alpha) { return GTR2(ndoth, alpha); }
float orc_hdr_pdf(const orc_scene* scene, const float* L, float env_angle) {
  orc_frame f; memset(&f, 0, sizeof(f)); f.env_angle = env_angle;
  Ctx C; C.s = scene; C.f = &f; memset(&C.c, 0, sizeof(C.c));
  return hdrPdf(C, vec3(L[0], L[1], L[2]), scene->hdr_resolution);
}
void orc_sample_hdr(const orc_scene* scene, float xi1, float xi2, float* L) {
  orc_frame f; memset(&f, 0, sizeof(f));
  Ctx C; C.s = scene; C.f = &f; memset(&C.c, 0, sizeof(C.c));
  vec3 v = SampleHdr(C, xi1, xi2);
  L[0] = v.x; L[1] = v.y; L[2] = v.z;
}
void orc_to_spherical(const float* L, float env_angle, float* uv) {
  orc_frame f; memset(&f, 0, sizeof(f)); f.env_angle = env_angle;
  orc_scene s; memset(&s, 0, sizeof(s));
  Ctx C; C.s = &s; C.f = &f;
  vec2 r = toSphericalCoord(C, vec3(L[0], L[1], L[2]));
  uv[0] = r.x; uv[1] = r.y;
}
// DisneyEval / DisneySample probes on a material given as Triangle_encoded texels 6..13
static Material material_from_texels(const float* t) {
  orc_scene s; memset(&s, 0, sizeof(s));
  float tri[14 * 3];
  memset(tri, 0, sizeof(tri));
  memcpy(tri + 18, t, sizeof(float) * 24);
  s.triangles = tri; s.n_triangles = 1;
  Ctx C; C.s = &s;
  return getMaterial(C, 0);
}
void orc_disney_eval(const float* mat_texels, const float* V, const float* N, const float* L, float* f_out,
                     float* pdf_out) {
  Material m = material_from_texels(mat_texels);
  float pdf;
  vec3 f = DisneyEval(m, vec3(V[0], V[1], V[2]), vec3(N[0], N[1], N[2]), vec3(L[0], L[1], L[2]), pdf);
  f_out[0] = f.x; f_out[1] = f.y; f_out[2] = f.z; *pdf_out = pdf;
}
void orc_disney_sample(const float* mat_texels, const float* xi, const float* V, const float* N, float* L_out,
                       float* f_out, float* pdf_out, int* is_refract) {
  Material m = material_from_texels(mat_texels);
  vec3 L; float pdf; bool refr;
  vec3 f = DisneySample(xi[0], xi[1], xi[2], m, vec3(V[0], V[1], V[2]), vec3(N[0], N[1], N[2]), L, pdf, refr);
  L_out[0] = L.x; L_out[1] = L.y; L_out[2] = L.z;
  f_out[0] = f.x; f_out[1] = f.y; f_out[2] = f.z; *pdf_out = pdf; *is_refract = refr ? 1 : 0;
}


// ------------------------------------------------------------------ display
// The presented image: with enableToneMapping the tone-mapping pass (TM:77-93: simpleACES
// TM:66-75, then pow(c, 1/2.2) with enableGammaCorrection), otherwise the screen blit
// (fragment_shader_screen.glsl:6-9); written to the 8-bit default framebuffer (GL unorm
// conversion round(clamp(c, 0, 1) * 255)) and saved by SaveFrame (Utility.h:19-30), which reads
// rows bottom-up and flips them, so out row 0 is the top of the image.
// frame: H x W x 3 floats, row 0 = bottom (the accumulation texture); flags: 1 tone map, 2 gamma.
static vec3 simpleACES(vec3 c) {  // TM:66-75
  const float a = 2.51f, b = 0.03f, y = 2.43f, d = 0.59f, e = 0.14f;
  vec3 num = c * (a * c + vec3(b));
  vec3 den = c * (y * c + vec3(d)) + vec3(e);
  vec3 r = num / den;
  return vec3(clamp_(r.x, 0.0f, 1.0f), clamp_(r.y, 0.0f, 1.0f), clamp_(r.z, 0.0f, 1.0f));
}
static uint8_t unorm8(float f) {
  f = clamp_(f, 0.0f, 1.0f);  // NaN -> 0 (fminf/fmaxf)
  return (uint8_t)(int)(f * 255.0f + 0.5f);
}
void orc_display(const float* frame, int W, int H, int flags, uint8_t* out) {
  for (int py = 0; py < H; py++)
    for (int px = 0; px < W; px++) {
      const float* p = frame + 3 * ((size_t)py * W + px);
      vec3 c(p[0], p[1], p[2]);
      if (flags & 1) {
        c = simpleACES(c);
        if (flags & 2) {
          const float g = 1.0f / 2.2f;
          c = vec3(pow_(c.x, g), pow_(c.y, g), pow_(c.z, g));
        }
      }
      uint8_t* o = out + 3 * ((size_t)(H - 1 - py) * W + px);
      o[0] = unorm8(c.x); o[1] = unorm8(c.y); o[2] = unorm8(c.z);
    }
}
}  // extern "C"
