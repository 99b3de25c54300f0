// rt_scene.cpp — host-side scene preparation for the MI355X path tracer (CPU, C++17).
//
// Re-implements the reference's host pipeline that produces the path tracer's inputs
// (see include/rt_scene.h for the function-by-function map).  Arithmetic follows the
// reference's fp32 evaluation order (glm 0.9.8 operator forms, std::sort comparators,
// the double-precision luminance of Utility.h) so that a build with the same libstdc++
// reproduces the reference's BVH node arrays bit for bit.  Compiled with
// -ffp-contract=off (no FMA contraction, as the reference's x86-64 SSE build).
#include "rt_scene.h"
#include "tri_filter.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <string>
#include <thread>
#include <vector>

namespace {

// ------------------------------------------------------------------- glm-style fp32 math
struct v3 {
  float x, y, z;
};
struct v4 {
  float x, y, z, w;
};
inline v3 mk(float x, float y, float z) { return v3{x, y, z}; }
inline v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
inline v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
inline v3 mul(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
inline v3 mulv(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
inline float dot3(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
// glm::cross (glm/detail/func_geometric.inl)
inline v3 cross3(v3 x, v3 y) { return mk(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y); }
// glm::normalize = v * inversesqrt(dot(v, v)), inversesqrt = 1 / sqrt
inline v3 normalize3(v3 v) { return mul(v, 1.0f / sqrtf(dot3(v, v))); }
// glm::min / glm::max for scalars (glm/detail/func_common.inl, 0.9.8)
inline float gmin(float x, float y) { return x < y ? x : y; }
inline float gmax(float x, float y) { return x > y ? x : y; }

// column-major mat4 as glm::mat4 (m[c] is column c)
struct m4 {
  v4 c[4];
};
inline v4 v4add(v4 a, v4 b) { return v4{a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }
inline v4 v4mul(v4 a, float s) { return v4{a.x * s, a.y * s, a.z * s, a.w * s}; }
m4 identity() {
  m4 m;
  for (int i = 0; i < 4; i++) m.c[i] = v4{0, 0, 0, 0};
  m.c[0].x = m.c[1].y = m.c[2].z = m.c[3].w = 1.0f;
  return m;
}
// glm 0.9.8 operator*(mat4, vec4): (m0*v0 + m1*v1) + (m2*v2 + m3*v3)
v4 mat_vec(const m4& m, v4 v) {
  v4 add0 = v4add(v4mul(m.c[0], v.x), v4mul(m.c[1], v.y));
  v4 add1 = v4add(v4mul(m.c[2], v.z), v4mul(m.c[3], v.w));
  return v4add(add0, add1);
}
// glm 0.9.8 operator*(mat4, mat4): Result[i] = A0*B[i][0] + A1*B[i][1] + A2*B[i][2] + A3*B[i][3]
m4 mat_mat(const m4& a, const m4& b) {
  m4 r;
  for (int i = 0; i < 4; i++) {
    v4 s = v4add(v4add(v4add(v4mul(a.c[0], b.c[i].x), v4mul(a.c[1], b.c[i].y)), v4mul(a.c[2], b.c[i].z)),
                 v4mul(a.c[3], b.c[i].w));
    r.c[i] = s;
  }
  return r;
}
// glm::scale(m, v)
m4 gscale(const m4& m, v3 v) {
  m4 r;
  r.c[0] = v4mul(m.c[0], v.x);
  r.c[1] = v4mul(m.c[1], v.y);
  r.c[2] = v4mul(m.c[2], v.z);
  r.c[3] = m.c[3];
  return r;
}
// glm::translate(m, v): Result[3] = m[0]*v[0] + m[1]*v[1] + m[2]*v[2] + m[3]
m4 gtranslate(const m4& m, v3 v) {
  m4 r = m;
  r.c[3] = v4add(v4add(v4add(v4mul(m.c[0], v.x), v4mul(m.c[1], v.y)), v4mul(m.c[2], v.z)), m.c[3]);
  return r;
}
// glm::rotate(m, angle, axis) (glm/gtc/matrix_transform.inl, 0.9.8)
m4 grotate(const m4& m, float angle, v3 v) {
  float a = angle;
  float c = cosf(a);
  float s = sinf(a);
  v3 axis = normalize3(v);
  v3 temp = mul(axis, 1.0f - c);
  float R[3][3];
  R[0][0] = c + temp.x * axis.x;
  R[0][1] = temp.x * axis.y + s * axis.z;
  R[0][2] = temp.x * axis.z - s * axis.y;
  R[1][0] = temp.y * axis.x - s * axis.z;
  R[1][1] = c + temp.y * axis.y;
  R[1][2] = temp.y * axis.z + s * axis.x;
  R[2][0] = temp.z * axis.x + s * axis.y;
  R[2][1] = temp.z * axis.y - s * axis.x;
  R[2][2] = c + temp.z * axis.z;
  m4 r;
  for (int i = 0; i < 3; i++)
    r.c[i] = v4add(v4add(v4mul(m.c[0], R[i][0]), v4mul(m.c[1], R[i][1])), v4mul(m.c[2], R[i][2]));
  r.c[3] = m.c[3];
  return r;
}
inline float radians(float deg) { return deg * 0.01745329251994329576923690768489f; }

// getTransformMatrix (src/core/Model.h:250-266): translate * rotate * scale
m4 transform_matrix(v3 rot, v3 tr, v3 sc) {
  m4 unit = identity();
  m4 scale = gscale(unit, sc);
  m4 translate = gtranslate(unit, tr);
  m4 rotate = unit;
  rotate = grotate(rotate, radians(rot.x), mk(1, 0, 0));
  rotate = grotate(rotate, radians(rot.y), mk(0, 1, 0));
  rotate = grotate(rotate, radians(rot.z), mk(0, 0, 1));
  return mat_mat(mat_mat(translate, rotate), scale);
}

// ------------------------------------------------------------------------ OBJ parse
// assimp's fast_atoreal_move<float> (code/Common/fast_atof.h): integer part as uint64 ->
// float, fraction as uint64 (<=15 digits) * 10^-n in double added in float, exponent
// applied as f *= powf(10, e).
const double kFastAtofTable[16] = {0.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001, 0.00000001,
                                   0.000000001, 0.0000000001, 0.00000000001, 0.000000000001, 0.0000000000001,
                                   0.00000000000001, 0.000000000000001};
uint64_t strtoul10_64(const char* in, const char** out, unsigned int* max_inout) {
  unsigned int cur = 0;
  uint64_t value = 0;
  while (*in >= '0' && *in <= '9') {
    value = value * 10 + (uint64_t)(*in - '0');
    ++in;
    ++cur;
    if (max_inout && *max_inout == cur) {
      while (*in >= '0' && *in <= '9') ++in;  // skip the remaining digits
      break;
    }
  }
  if (out) *out = in;
  if (max_inout) *max_inout = cur;
  return value;
}
const char* fast_atof_assimp(const char* c, float& out) {
  float f = 0;
  bool inv = (*c == '-');
  if (inv || *c == '+') ++c;
  if (!(c[0] >= '0' && c[0] <= '9') && !(c[0] == '.' && c[1] >= '0' && c[1] <= '9')) {
    out = 0;
    return nullptr;
  }
  if (*c != '.') f = (float)strtoul10_64(c, &c, nullptr);
  if (*c == '.' && c[1] >= '0' && c[1] <= '9') {
    ++c;
    unsigned int diff = 15;
    double pl = (double)strtoul10_64(c, &c, &diff);
    pl *= kFastAtofTable[diff];
    f += (float)pl;
  } else if (*c == '.') {
    ++c;
  }
  if (*c == 'e' || *c == 'E') {
    ++c;
    bool einv = (*c == '-');
    if (einv || *c == '+') ++c;
    float e = (float)strtoul10_64(c, &c, nullptr);
    if (einv) e = -e;
    f *= powf(10.0f, e);
  }
  if (inv) f = -f;
  out = f;
  return c;
}

struct RawObj {
  std::vector<float> pos, nrm;
  std::vector<int32_t> face_sizes, pidx, nidx;
};

inline const char* skip_ws(const char* p) {
  while (*p == ' ' || *p == '\t') ++p;
  return p;
}

int parse_obj(const char* path, int mode, RawObj& raw) {
  FILE* fp = fopen(path, "rb");
  if (!fp) return RTS_ERR_IO;
  std::string text;
  char buf[1 << 16];
  size_t n;
  while ((n = fread(buf, 1, sizeof(buf), fp)) > 0) text.append(buf, n);
  fclose(fp);
  const char* p = text.c_str();
  const char* end = p + text.size();
  auto parse_float = [&](const char* q, float& v) -> const char* {
    q = skip_ws(q);
    if (mode == 0) {
      char* e = nullptr;
      v = strtof(q, &e);
      return (e == q) ? nullptr : e;
    }
    return fast_atof_assimp(q, v);
  };
  while (p < end) {
    const char* line = skip_ws(p);
    const char* eol = (const char*)memchr(line, '\n', (size_t)(end - line));
    if (!eol) eol = end;
    if (line[0] == 'v' && (line[1] == ' ' || line[1] == '\t')) {
      float v[3] = {0, 0, 0};
      const char* q = line + 1;
      for (int k = 0; k < 3 && q; k++) q = parse_float(q, v[k]);
      if (!q) return RTS_ERR_FORMAT;
      raw.pos.insert(raw.pos.end(), v, v + 3);
    } else if (line[0] == 'v' && line[1] == 'n' && (line[2] == ' ' || line[2] == '\t')) {
      float v[3] = {0, 0, 0};
      const char* q = line + 2;
      for (int k = 0; k < 3 && q; k++) q = parse_float(q, v[k]);
      if (!q) return RTS_ERR_FORMAT;
      raw.nrm.insert(raw.nrm.end(), v, v + 3);
    } else if (line[0] == 'f' && (line[1] == ' ' || line[1] == '\t')) {
      const char* q = line + 1;
      int count = 0;
      while (true) {
        q = skip_ws(q);
        if (q >= eol || *q == '\r' || *q == '\n' || *q == '#') break;
        char* e = nullptr;
        long vi = strtol(q, &e, 10);
        if (e == q) return RTS_ERR_FORMAT;
        q = e;
        long ti = 0, ni = 0;
        if (*q == '/') {
          ++q;
          if (*q != '/') { ti = strtol(q, &e, 10); q = e; }
          if (*q == '/') { ++q; ni = strtol(q, &e, 10); q = e; }
        }
        (void)ti;
        int npos = (int)(raw.pos.size() / 3), nnrm = (int)(raw.nrm.size() / 3);
        long rv = vi > 0 ? vi - 1 : npos + vi;     // negative = relative (OBJ spec)
        long rn = ni > 0 ? ni - 1 : (ni < 0 ? nnrm + ni : -1);
        if (rv < 0 || rv >= npos) return RTS_ERR_FORMAT;
        if (rn >= nnrm) return RTS_ERR_FORMAT;
        raw.pidx.push_back((int32_t)rv);
        raw.nidx.push_back((int32_t)rn);
        count++;
      }
      if (count > 0) raw.face_sizes.push_back(count);
    }
    p = eol + 1;
  }
  return RTS_OK;
}

}  // namespace

// ---------------------------------------------------------------------- mesh (assimp)
struct rts_mesh {
  std::vector<v3> pos;      // corner vertices (unshared), assimp ObjFileImporter::createVertexArray
  std::vector<v3> nrm;
  std::vector<int32_t> idx; // triangle list after aiProcess_Triangulate
};

namespace {

// assimp SpatialSort (code/Common/SpatialSort.cpp, 5.2): entries sorted by signed distance
// of (p - centroid) to a fixed plane; FindPositions returns matches in that order.
struct SpatialSort {
  struct Entry {
    unsigned int idx;
    v3 p;
    float d;
    bool operator<(const Entry& o) const { return d < o.d; }
  };
  v3 normal, centroid;
  std::vector<Entry> e;
  float dist(v3 p) const { return dot3(sub(p, centroid), normal); }
  void fill(const std::vector<v3>& pts) {
    normal = mk(0.8523f, 0.0005f, 0.5229f);
    normal = mul(normal, 1.0f / sqrtf(dot3(normal, normal)));  // aiVector3D::Normalize
    e.resize(pts.size());
    for (size_t i = 0; i < pts.size(); i++) e[i] = Entry{(unsigned)i, pts[i], 0.0f};
    centroid = mk(0, 0, 0);
    float scale = 1.0f / (float)pts.size();
    for (size_t i = 0; i < pts.size(); i++) centroid = add(centroid, mul(pts[i], scale));
    for (size_t i = 0; i < e.size(); i++) e[i].d = dist(e[i].p);
    std::sort(e.begin(), e.end());
  }
  void find(v3 p, float radius, std::vector<unsigned>& out) const {
    out.clear();
    float d = dist(p);
    float minD = d - radius, maxD = d + radius;
    if (e.empty() || maxD < e.front().d || minD > e.back().d) return;
    unsigned index = (unsigned)e.size() / 2;
    unsigned step = (unsigned)e.size() / 4;
    while (step > 1) {
      if (e[index].d < minD) index += step;
      else index -= step;
      step /= 2;
    }
    while (index > 0 && e[index].d > minD) index--;
    while (index < e.size() - 1 && e[index].d < minD) index++;
    float sq = radius * radius;
    for (size_t it = index; it < e.size() && e[it].d < maxD; ++it) {
      v3 df = sub(e[it].p, p);
      if (dot3(df, df) < sq) out.push_back(e[it].idx);
    }
  }
};

// aiVector3D::NormalizeSafe (x *= 1/len when len > 0)
inline v3 normalize_safe(v3 v) {
  float len = sqrtf(dot3(v, v));
  if (len > 0.0f) {
    float inv = 1.0f / len;
    v = mk(v.x * inv, v.y * inv, v.z * inv);
  }
  return v;
}

int build_mesh(const RawObj& raw, rts_mesh*& out) {
  rts_mesh* m = new (std::nothrow) rts_mesh();
  if (!m) return RTS_ERR_NOMEM;
  bool has_normals = !raw.nrm.empty();
  for (int32_t k : raw.nidx)
    if (k < 0) has_normals = false;
  // unshared corner vertices in face order
  size_t cursor = 0;
  for (size_t f = 0; f < raw.face_sizes.size(); f++) {
    int fs = raw.face_sizes[f];
    int base = (int)m->pos.size();
    for (int k = 0; k < fs; k++) {
      int pi = raw.pidx[cursor + k];
      m->pos.push_back(mk(raw.pos[3 * pi], raw.pos[3 * pi + 1], raw.pos[3 * pi + 2]));
      if (has_normals) {
        int ni = raw.nidx[cursor + k];
        m->nrm.push_back(mk(raw.nrm[3 * ni], raw.nrm[3 * ni + 1], raw.nrm[3 * ni + 2]));
      }
    }
    cursor += fs;
    // aiProcess_Triangulate (code/PostProcessing/TriangulateProcess.cpp)
    if (fs < 3) continue;  // points/lines carry no triangles
    if (fs == 3) {
      m->idx.push_back(base); m->idx.push_back(base + 1); m->idx.push_back(base + 2);
    } else if (fs == 4) {
      int start = 0;
      for (int i = 0; i < 4; ++i) {  // the concave corner (if any) starts the fan
        v3 v0 = m->pos[base + (i + 3) % 4], v1 = m->pos[base + (i + 2) % 4];
        v3 v2 = m->pos[base + (i + 1) % 4], v = m->pos[base + i];
        v3 left = normalize_safe(sub(v0, v)), diag = normalize_safe(sub(v1, v)), right = normalize_safe(sub(v2, v));
        float angle = acosf(dot3(left, diag)) + acosf(dot3(right, diag));
        if (angle > 3.14159265358979323846f) { start = i; break; }
      }
      int t[4] = {base, base + 1, base + 2, base + 3};
      m->idx.push_back(t[start]); m->idx.push_back(t[(start + 1) % 4]); m->idx.push_back(t[(start + 2) % 4]);
      m->idx.push_back(t[start]); m->idx.push_back(t[(start + 2) % 4]); m->idx.push_back(t[(start + 3) % 4]);
    } else {
      // convex n-gon: triangle fan (assimp ear-clips; none of the shipped assets has n > 4)
      for (int k = 1; k + 1 < fs; k++) {
        m->idx.push_back(base); m->idx.push_back(base + k); m->idx.push_back(base + k + 1);
      }
    }
  }
  if (!has_normals) {
    // aiProcess_GenSmoothNormals (code/PostProcessing/GenVertexNormalsProcess.cpp), default
    // max angle 175 deg -> the "no angle limit" branch: every vertex within the position
    // epsilon receives the normalised sum of the (normalised) face normals found.
    size_t nv = m->pos.size();
    std::vector<v3> fn(nv, mk(NAN, NAN, NAN));
    // face normals over the *original polygons* (assimp computes them after triangulation:
    // each triangle writes its own normal to its three corners)
    for (size_t t = 0; t + 2 < m->idx.size(); t += 3) {
      v3 p1 = m->pos[m->idx[t]], p2 = m->pos[m->idx[t + 1]], p3 = m->pos[m->idx[t + 2]];
      v3 a = sub(p2, p1), b = sub(p3, p1);
      v3 c = mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);  // aiVector3D operator^
      v3 n = normalize_safe(c);
      fn[m->idx[t]] = n; fn[m->idx[t + 1]] = n; fn[m->idx[t + 2]] = n;
    }
    // ComputePositionEpsilon: |max - min| * 1e-4
    v3 mn = mk(1e10f, 1e10f, 1e10f), mx = mk(-1e10f, -1e10f, -1e10f);
    for (const v3& p : m->pos) {
      mn = mk(std::min(mn.x, p.x), std::min(mn.y, p.y), std::min(mn.z, p.z));
      mx = mk(std::max(mx.x, p.x), std::max(mx.y, p.y), std::max(mx.z, p.z));
    }
    v3 diag = sub(mx, mn);
    float eps = sqrtf(dot3(diag, diag)) * 1e-4f;
    SpatialSort ss;
    ss.fill(m->pos);
    std::vector<v3> out(nv, mk(0, 0, 0));
    std::vector<bool> had(nv, false);
    std::vector<unsigned> found;
    for (size_t i = 0; i < nv; i++) {
      if (had[i]) continue;
      ss.find(m->pos[i], eps, found);
      v3 s = mk(0, 0, 0);
      for (unsigned k : found) {
        v3 v = fn[k];
        if (!(v.x != v.x)) s = add(s, v);
      }
      s = normalize_safe(s);
      for (unsigned k : found) {
        out[k] = s;
        had[k] = true;
      }
    }
    m->nrm.swap(out);
  }
  out = m;
  return RTS_OK;
}

// ------------------------------------------------------------------------ scene / BVH
struct Tri {
  v3 p1, p2, p3, n1, n2, n3;
  int32_t mat;  // index into the scene's material list
  int32_t src;  // pre-BVH index
};
struct Node {
  int left, right, n, index;
  v3 AA, BB;
};

const float kINF = 114514.0f;  // src/core/BVH.h:8

// cmpx/cmpy/cmpz (src/core/BVH.h:24-40): centre = (p1 + p2 + p3) / vec3(3)
inline float centre(const Tri& t, int axis) {
  v3 c = add(add(t.p1, t.p2), t.p3);
  c = mk(c.x / 3.0f, c.y / 3.0f, c.z / 3.0f);
  return axis == 0 ? c.x : (axis == 1 ? c.y : c.z);
}
bool cmpx(const Tri& a, const Tri& b) { return centre(a, 0) < centre(b, 0); }
bool cmpy(const Tri& a, const Tri& b) { return centre(a, 1) < centre(b, 1); }
bool cmpz(const Tri& a, const Tri& b) { return centre(a, 2) < centre(b, 2); }

inline float min3(float a, float b, float c) { return gmin(a, gmin(b, c)); }
inline float max3(float a, float b, float c) { return gmax(a, gmax(b, c)); }

// buildBVHwithSAH (src/core/BVH.h:110-241), literal restatement.
int build_sah(std::vector<Tri>& tris, std::vector<Node>& nodes, int l, int r, int n) {
  if (l > r) return 0;
  nodes.push_back(Node());
  int id = (int)nodes.size() - 1;
  nodes[id].left = nodes[id].right = nodes[id].n = nodes[id].index = 0;
  nodes[id].AA = mk(1145141919.0f, 1145141919.0f, 1145141919.0f);
  nodes[id].BB = mk(-1145141919.0f, -1145141919.0f, -1145141919.0f);
  for (int i = l; i <= r; i++) {
    const Tri& t = tris[i];
    float minx = gmin(t.p1.x, gmin(t.p2.x, t.p3.x));
    float miny = gmin(t.p1.y, gmin(t.p2.y, t.p3.y));
    float minz = gmin(t.p1.z, gmin(t.p2.z, t.p3.z));
    nodes[id].AA.x = gmin(nodes[id].AA.x, minx);
    nodes[id].AA.y = gmin(nodes[id].AA.y, miny);
    nodes[id].AA.z = gmin(nodes[id].AA.z, minz);
    float maxx = gmax(t.p1.x, gmax(t.p2.x, t.p3.x));
    float maxy = gmax(t.p1.y, gmax(t.p2.y, t.p3.y));
    float maxz = gmax(t.p1.z, gmax(t.p2.z, t.p3.z));
    nodes[id].BB.x = gmax(nodes[id].BB.x, maxx);
    nodes[id].BB.y = gmax(nodes[id].BB.y, maxy);
    nodes[id].BB.z = gmax(nodes[id].BB.z, maxz);
  }
  if ((r - l + 1) <= n) {
    nodes[id].n = r - l + 1;
    nodes[id].index = l;
    return id;
  }
  float Cost = kINF;
  int Axis = 0;
  int Split = (l + r) / 2;
  int cnt = r - l + 1;
  std::vector<v3> leftMax(cnt), leftMin(cnt), rightMax(cnt), rightMin(cnt);
  for (int axis = 0; axis < 3; axis++) {
    if (axis == 0) std::sort(&tris[0] + l, &tris[0] + r + 1, cmpx);
    if (axis == 1) std::sort(&tris[0] + l, &tris[0] + r + 1, cmpy);
    if (axis == 2) std::sort(&tris[0] + l, &tris[0] + r + 1, cmpz);
    for (int k = 0; k < cnt; k++) {
      leftMax[k] = mk(-kINF, -kINF, -kINF);
      leftMin[k] = mk(kINF, kINF, kINF);
      rightMax[k] = mk(-kINF, -kINF, -kINF);
      rightMin[k] = mk(kINF, kINF, kINF);
    }
    for (int i = l; i <= r; i++) {
      const Tri& t = tris[i];
      int bias = (i == l) ? 0 : 1;
      leftMax[i - l].x = gmax(leftMax[i - l - bias].x, max3(t.p1.x, t.p2.x, t.p3.x));
      leftMax[i - l].y = gmax(leftMax[i - l - bias].y, max3(t.p1.y, t.p2.y, t.p3.y));
      leftMax[i - l].z = gmax(leftMax[i - l - bias].z, max3(t.p1.z, t.p2.z, t.p3.z));
      leftMin[i - l].x = gmin(leftMin[i - l - bias].x, min3(t.p1.x, t.p2.x, t.p3.x));
      leftMin[i - l].y = gmin(leftMin[i - l - bias].y, min3(t.p1.y, t.p2.y, t.p3.y));
      leftMin[i - l].z = gmin(leftMin[i - l - bias].z, min3(t.p1.z, t.p2.z, t.p3.z));
    }
    for (int i = r; i >= l; i--) {
      const Tri& t = tris[i];
      int bias = (i == r) ? 0 : 1;
      rightMax[i - l].x = gmax(rightMax[i - l + bias].x, max3(t.p1.x, t.p2.x, t.p3.x));
      rightMax[i - l].y = gmax(rightMax[i - l + bias].y, max3(t.p1.y, t.p2.y, t.p3.y));
      rightMax[i - l].z = gmax(rightMax[i - l + bias].z, max3(t.p1.z, t.p2.z, t.p3.z));
      rightMin[i - l].x = gmin(rightMin[i - l + bias].x, min3(t.p1.x, t.p2.x, t.p3.x));
      rightMin[i - l].y = gmin(rightMin[i - l + bias].y, min3(t.p1.y, t.p2.y, t.p3.y));
      rightMin[i - l].z = gmin(rightMin[i - l + bias].z, min3(t.p1.z, t.p2.z, t.p3.z));
    }
    float cost = kINF;
    int split = l;
    for (int i = l; i <= r - 1; i++) {
      float lenx, leny, lenz;
      v3 leftAA = leftMin[i - l], leftBB = leftMax[i - l];
      lenx = leftBB.x - leftAA.x;
      leny = leftBB.y - leftAA.y;
      lenz = leftBB.z - leftAA.z;
      float leftS = (float)(2.0 * (double)((lenx * leny) + (lenx * lenz) + (leny * lenz)));
      float leftCost = leftS * (float)(i - l + 1);
      v3 rightAA = rightMin[i + 1 - l], rightBB = rightMax[i + 1 - l];
      lenx = rightBB.x - rightAA.x;
      leny = rightBB.y - rightAA.y;
      lenz = rightBB.z - rightAA.z;
      float rightS = (float)(2.0 * (double)((lenx * leny) + (lenx * lenz) + (leny * lenz)));
      float rightCost = rightS * (float)(r - i);
      float totalCost = leftCost + rightCost;
      if (totalCost < cost) {
        cost = totalCost;
        split = i;
      }
    }
    if (cost < Cost) {  // R18: nodes whose best cost >= 114514 keep the X-median split
      Cost = cost;
      Axis = axis;
      Split = split;
    }
  }
  if (Axis == 0) std::sort(&tris[0] + l, &tris[0] + r + 1, cmpx);
  if (Axis == 1) std::sort(&tris[0] + l, &tris[0] + r + 1, cmpy);
  if (Axis == 2) std::sort(&tris[0] + l, &tris[0] + r + 1, cmpz);
  int left = build_sah(tris, nodes, l, Split, n);
  int right = build_sah(tris, nodes, Split + 1, r, n);
  nodes[id].left = left;
  nodes[id].right = right;
  return id;
}

// The same build, faster and with identical output ("faithful" mode):
// * the per-axis std::sort runs on a 4-byte index permutation compared through precomputed
//   centroids (the same (p1+p2+p3)/3 fp32 values); libstdc++'s introsort does the same
//   comparisons and moves whatever the element type, so the permutation is identical;
// * prefix/suffix boxes read precomputed per-triangle bounds (the same min3/max3 values);
// * subtrees over disjoint triangle ranges are built concurrently into local node vectors and
//   spliced back in the reference's pre-order numbering.
struct FastBuild {
  std::vector<float> c[3];      // centroid per triangle and axis
  std::vector<v3> tmin, tmax;   // per-triangle bounds
  std::vector<int32_t> perm;    // current triangle order (indices into the input array)
  int n;
  int par_depth;
};

void fast_sort(FastBuild& B, int l, int r, int axis) {
  const float* key = B.c[axis].data();
  std::sort(B.perm.data() + l, B.perm.data() + r + 1, [key](int32_t a, int32_t b) { return key[a] < key[b]; });
}

// appends the subtree over [l, r] to `nodes` in pre-order (local ids); returns its root id
int fast_sah(FastBuild& B, std::vector<Node>& nodes, int l, int r, int depth) {
  if (l > r) return 0;
  nodes.push_back(Node());
  const int id = (int)nodes.size() - 1;
  Node nd;
  nd.left = nd.right = nd.n = nd.index = 0;
  nd.AA = mk(1145141919.0f, 1145141919.0f, 1145141919.0f);
  nd.BB = mk(-1145141919.0f, -1145141919.0f, -1145141919.0f);
  for (int i = l; i <= r; i++) {
    const int t = B.perm[i];
    nd.AA.x = gmin(nd.AA.x, B.tmin[t].x); nd.AA.y = gmin(nd.AA.y, B.tmin[t].y); nd.AA.z = gmin(nd.AA.z, B.tmin[t].z);
    nd.BB.x = gmax(nd.BB.x, B.tmax[t].x); nd.BB.y = gmax(nd.BB.y, B.tmax[t].y); nd.BB.z = gmax(nd.BB.z, B.tmax[t].z);
  }
  if ((r - l + 1) <= B.n) {
    nd.n = r - l + 1;
    nd.index = l;
    nodes[id] = nd;
    return id;
  }
  float Cost = kINF;
  int Axis = 0, Split = (l + r) / 2;
  const int cnt = r - l + 1;
  std::vector<v3> leftMax(cnt), leftMin(cnt), rightMax(cnt), rightMin(cnt);
  for (int axis = 0; axis < 3; axis++) {
    fast_sort(B, l, r, axis);
    for (int i = l; i <= r; i++) {  // BVH.h:158-168 (the kINF initialisers are overwritten)
      const int t = B.perm[i];
      const int k = i - l, kp = (i == l) ? k : k - 1;
      const v3 pmax = (i == l) ? mk(-kINF, -kINF, -kINF) : leftMax[kp], pmin = (i == l) ? mk(kINF, kINF, kINF) : leftMin[kp];
      leftMax[k] = mk(gmax(pmax.x, B.tmax[t].x), gmax(pmax.y, B.tmax[t].y), gmax(pmax.z, B.tmax[t].z));
      leftMin[k] = mk(gmin(pmin.x, B.tmin[t].x), gmin(pmin.y, B.tmin[t].y), gmin(pmin.z, B.tmin[t].z));
    }
    for (int i = r; i >= l; i--) {
      const int t = B.perm[i];
      const int k = i - l, kp = (i == r) ? k : k + 1;
      const v3 pmax = (i == r) ? mk(-kINF, -kINF, -kINF) : rightMax[kp], pmin = (i == r) ? mk(kINF, kINF, kINF) : rightMin[kp];
      rightMax[k] = mk(gmax(pmax.x, B.tmax[t].x), gmax(pmax.y, B.tmax[t].y), gmax(pmax.z, B.tmax[t].z));
      rightMin[k] = mk(gmin(pmin.x, B.tmin[t].x), gmin(pmin.y, B.tmin[t].y), gmin(pmin.z, B.tmin[t].z));
    }
    float cost = kINF;
    int split = l;
    for (int i = l; i <= r - 1; i++) {
      const v3 leftAA = leftMin[i - l], leftBB = leftMax[i - l];
      float lenx = leftBB.x - leftAA.x, leny = leftBB.y - leftAA.y, lenz = leftBB.z - leftAA.z;
      const float leftS = (float)(2.0 * (double)((lenx * leny) + (lenx * lenz) + (leny * lenz)));
      const float leftCost = leftS * (float)(i - l + 1);
      const v3 rightAA = rightMin[i + 1 - l], rightBB = rightMax[i + 1 - l];
      lenx = rightBB.x - rightAA.x; leny = rightBB.y - rightAA.y; lenz = rightBB.z - rightAA.z;
      const float rightS = (float)(2.0 * (double)((lenx * leny) + (lenx * lenz) + (leny * lenz)));
      const float rightCost = rightS * (float)(r - i);
      const float totalCost = leftCost + rightCost;
      if (totalCost < cost) { cost = totalCost; split = i; }
    }
    if (cost < Cost) { Cost = cost; Axis = axis; Split = split; }
  }
  fast_sort(B, l, r, Axis);
  std::vector<v3>().swap(leftMax); std::vector<v3>().swap(leftMin);
  std::vector<v3>().swap(rightMax); std::vector<v3>().swap(rightMin);
  int left, right;
  if (depth < B.par_depth && cnt > 4096) {
    // the two subtrees own disjoint ranges of perm: build them concurrently, then splice
    std::vector<Node> ln, rn;
    std::thread th([&] { fast_sah(B, ln, l, Split, depth + 1); });
    fast_sah(B, rn, Split + 1, r, depth + 1);
    th.join();
    auto splice = [&](std::vector<Node>& sub) {
      if (sub.empty()) return 0;
      const int base = (int)nodes.size();
      for (Node& x : sub) {
        if (x.n == 0) { x.left += base; x.right += base; }  // internal: children are local ids >= 1
        nodes.push_back(x);
      }
      return base;
    };
    left = splice(ln);
    right = splice(rn);
  } else {
    left = fast_sah(B, nodes, l, Split, depth + 1);
    right = fast_sah(B, nodes, Split + 1, r, depth + 1);
  }
  nd.left = left;
  nd.right = right;
  nodes[id] = nd;
  return id;
}

void build_sah_fast(std::vector<Tri>& tris, std::vector<Node>& nodes, int n) {
  const int nt = (int)tris.size();
  FastBuild B;
  B.n = n;
  unsigned hw = std::thread::hardware_concurrency();
  B.par_depth = 0;
  while ((1u << B.par_depth) < std::max(1u, hw) * 2u && B.par_depth < 6) B.par_depth++;
  for (int a = 0; a < 3; a++) B.c[a].resize(nt);
  B.tmin.resize(nt); B.tmax.resize(nt); B.perm.resize(nt);
  for (int t = 0; t < nt; t++) {
    const Tri& x = tris[t];
    B.c[0][t] = centre(x, 0); B.c[1][t] = centre(x, 1); B.c[2][t] = centre(x, 2);
    B.tmin[t] = mk(min3(x.p1.x, x.p2.x, x.p3.x), min3(x.p1.y, x.p2.y, x.p3.y), min3(x.p1.z, x.p2.z, x.p3.z));
    B.tmax[t] = mk(max3(x.p1.x, x.p2.x, x.p3.x), max3(x.p1.y, x.p2.y, x.p3.y), max3(x.p1.z, x.p2.z, x.p3.z));
    B.perm[t] = t;
  }
  std::vector<Node> local;
  local.reserve(2 * (size_t)nt / std::max(1, n) + 2);
  fast_sah(B, local, 0, nt - 1, 0);
  const int base = (int)nodes.size();  // after the dummy node 0
  for (Node& x : local) {
    if (x.n == 0) { x.left += base; x.right += base; }
    nodes.push_back(x);
  }
  std::vector<Tri> sorted(nt);
  for (int i = 0; i < nt; i++) sorted[i] = tris[B.perm[i]];
  tris.swap(sorted);
}

void tree_stats(const std::vector<Node>& nodes, int root, int32_t& depth, int32_t& leaves) {
  depth = 0;
  leaves = 0;
  if (root <= 0 || root >= (int)nodes.size()) return;
  std::vector<std::pair<int, int>> st;
  st.push_back({root, 1});  // depth counted in levels (root = 1), as SURVEY.md §8(a)
  while (!st.empty()) {
    auto e = st.back();
    st.pop_back();
    const Node& nd = nodes[e.first];
    if (e.second > depth) depth = e.second;
    if (nd.n > 0) {
      leaves++;
      continue;
    }
    if (nd.left > 0) st.push_back({nd.left, e.second + 1});
    if (nd.right > 0) st.push_back({nd.right, e.second + 1});
  }
}

}  // namespace

struct rts_scene {
  std::vector<Tri> tris;
  std::vector<rts_material> mats;
  std::vector<Node> nodes;  // empty until build; node 0 = the dummy of src/core/Scene.h:189-195
  bool built = false;
};

namespace {
bool same_material(const rts_material& a, const rts_material& b) { return memcmp(&a, &b, sizeof(a)) == 0; }
int add_material(rts_scene* s, const rts_material& m) {
  for (size_t i = 0; i < s->mats.size(); i++)
    if (same_material(s->mats[i], m)) return (int)i;
  s->mats.push_back(m);
  return (int)s->mats.size() - 1;
}
}  // namespace

extern "C" {

int rts_obj_parse_raw(const char* path, int parse_mode, int32_t* n_positions, int32_t* n_normals, int32_t* n_faces,
                      int32_t* n_indices, float* positions, float* normals, int32_t* face_sizes, int32_t* pos_index,
                      int32_t* nrm_index) {
  if (!path || !n_positions || !n_normals || !n_faces || !n_indices) return RTS_ERR_ARG;
  RawObj raw;
  int rc = parse_obj(path, parse_mode, raw);
  if (rc) return rc;
  *n_positions = (int32_t)(raw.pos.size() / 3);
  *n_normals = (int32_t)(raw.nrm.size() / 3);
  *n_faces = (int32_t)raw.face_sizes.size();
  *n_indices = (int32_t)raw.pidx.size();
  if (positions) memcpy(positions, raw.pos.data(), raw.pos.size() * sizeof(float));
  if (normals) memcpy(normals, raw.nrm.data(), raw.nrm.size() * sizeof(float));
  if (face_sizes) memcpy(face_sizes, raw.face_sizes.data(), raw.face_sizes.size() * sizeof(int32_t));
  if (pos_index) memcpy(pos_index, raw.pidx.data(), raw.pidx.size() * sizeof(int32_t));
  if (nrm_index) memcpy(nrm_index, raw.nidx.data(), raw.nidx.size() * sizeof(int32_t));
  return RTS_OK;
}

int rts_obj_load(const char* path, int parse_mode, rts_mesh** out) {
  if (!path || !out) return RTS_ERR_ARG;
  RawObj raw;
  int rc = parse_obj(path, parse_mode, raw);
  if (rc) return rc;
  return build_mesh(raw, *out);
}

int rts_mesh_from_raw(const float* positions, int n_positions, const float* normals, int n_normals,
                      const int32_t* face_sizes, int n_faces, const int32_t* pos_index, const int32_t* nrm_index,
                      rts_mesh** out) {
  if (!out || n_positions < 0 || n_faces < 0 || (n_positions && !positions) || (n_faces && (!face_sizes || !pos_index)))
    return RTS_ERR_ARG;
  RawObj raw;
  raw.pos.assign(positions, positions + 3 * (size_t)n_positions);
  if (normals && n_normals > 0) raw.nrm.assign(normals, normals + 3 * (size_t)n_normals);
  raw.face_sizes.assign(face_sizes, face_sizes + n_faces);
  size_t ni = 0;
  for (int f = 0; f < n_faces; f++) {
    if (face_sizes[f] < 0) return RTS_ERR_ARG;
    ni += (size_t)face_sizes[f];
  }
  raw.pidx.assign(pos_index, pos_index + ni);
  if (nrm_index) raw.nidx.assign(nrm_index, nrm_index + ni);
  else raw.nidx.assign(ni, -1);
  for (size_t k = 0; k < ni; k++) {
    if (raw.pidx[k] < 0 || raw.pidx[k] >= n_positions) return RTS_ERR_ARG;
    if (raw.nidx[k] >= n_normals) return RTS_ERR_ARG;
  }
  return build_mesh(raw, *out);
}

int rts_mesh_counts(const rts_mesh* m, int32_t* n_vertices, int32_t* n_indices) {
  if (!m) return RTS_ERR_ARG;
  if (n_vertices) *n_vertices = (int32_t)m->pos.size();
  if (n_indices) *n_indices = (int32_t)m->idx.size();
  return RTS_OK;
}

int rts_mesh_data(const rts_mesh* m, float* positions, float* normals, int32_t* indices) {
  if (!m) return RTS_ERR_ARG;
  for (size_t i = 0; i < m->pos.size(); i++) {
    if (positions) { positions[3 * i] = m->pos[i].x; positions[3 * i + 1] = m->pos[i].y; positions[3 * i + 2] = m->pos[i].z; }
    if (normals) { normals[3 * i] = m->nrm[i].x; normals[3 * i + 1] = m->nrm[i].y; normals[3 * i + 2] = m->nrm[i].z; }
  }
  if (indices) memcpy(indices, m->idx.data(), m->idx.size() * sizeof(int32_t));
  return RTS_OK;
}

void rts_mesh_free(rts_mesh* m) { delete m; }

int rts_scene_create(rts_scene** out) {
  if (!out) return RTS_ERR_ARG;
  *out = new (std::nothrow) rts_scene();
  return *out ? RTS_OK : RTS_ERR_NOMEM;
}

void rts_scene_free(rts_scene* s) { delete s; }

// getTriangle (src/core/Triangle.h:41-131), including the R17 normalisation bug.
int rts_scene_add_mesh(rts_scene* s, const rts_mesh* m, const rts_material* mat, const float rotate_deg[3],
                       const float translate[3], const float scale[3], int smooth_normal, int32_t range[2]) {
  if (!s || !m || !mat || !rotate_deg || !translate || !scale) return RTS_ERR_ARG;
  if (s->built) return RTS_ERR_STATE;
  m4 trans = transform_matrix(mk(rotate_deg[0], rotate_deg[1], rotate_deg[2]),
                              mk(translate[0], translate[1], translate[2]), mk(scale[0], scale[1], scale[2]));
  std::vector<v3> vertices = m->pos;
  std::vector<v3> normals = m->nrm;
  float maxx = -11451419.19f, maxy = -11451419.19f, maxz = -11451419.19f;
  float minx = 11451419.19f, miny = 11451419.19f, minz = 11451419.19f;
  for (const v3& p : m->pos) {
    maxx = gmax(maxx, p.x);
    maxy = gmax(maxx, p.y);  // R17: compares against maxx
    maxz = gmax(maxx, p.z);
    minx = gmin(minx, p.x);
    miny = gmin(minx, p.y);
    minz = gmin(minx, p.z);
  }
  float lenx = maxx - minx, leny = maxy - miny, lenz = maxz - minz;
  float maxaxis = gmax(lenx, gmax(leny, lenz));
  for (v3& v : vertices) { v.x /= maxaxis; v.y /= maxaxis; v.z /= maxaxis; }
  for (v3& v : vertices) {
    v4 vv = mat_vec(trans, v4{v.x, v.y, v.z, 1.0f});
    v = mk(vv.x, vv.y, vv.z);
  }
  for (v3& n : normals) {
    v4 nn = mat_vec(trans, v4{n.x, n.y, n.z, 0.0f});
    n = mk(nn.x, nn.y, nn.z);
  }
  int mid = add_material(s, *mat);
  int offset = (int)s->tris.size();
  size_t nt = m->idx.size() / 3;
  s->tris.resize(offset + nt);
  for (size_t i = 0; i < m->idx.size(); i += 3) {
    Tri& t = s->tris[offset + i / 3];
    t.p1 = vertices[m->idx[i]];
    t.p2 = vertices[m->idx[i + 1]];
    t.p3 = vertices[m->idx[i + 2]];
    if (!smooth_normal) {
      v3 n = normalize3(cross3(sub(t.p2, t.p1), sub(t.p3, t.p1)));
      t.n1 = t.n2 = t.n3 = n;
    } else {
      t.n1 = normalize3(normals[m->idx[i]]);
      t.n2 = normalize3(normals[m->idx[i + 1]]);
      t.n3 = normalize3(normals[m->idx[i + 2]]);
    }
    t.mat = mid;
    t.src = offset + (int)(i / 3);
  }
  if (range) { range[0] = offset; range[1] = (int32_t)s->tris.size(); }
  return RTS_OK;
}

int rts_scene_add_triangles(rts_scene* s, const float* positions, int n, const rts_material* mat, int32_t range[2]) {
  if (!s || !mat || n < 0 || (n && !positions)) return RTS_ERR_ARG;
  if (s->built) return RTS_ERR_STATE;
  int mid = add_material(s, *mat);
  int offset = (int)s->tris.size();
  s->tris.resize(offset + (size_t)n);
  for (int i = 0; i < n; i++) {
    Tri& t = s->tris[offset + i];
    const float* q = positions + 9 * (size_t)i;
    t.p1 = mk(q[0], q[1], q[2]);
    t.p2 = mk(q[3], q[4], q[5]);
    t.p3 = mk(q[6], q[7], q[8]);
    v3 nn = normalize3(cross3(sub(t.p2, t.p1), sub(t.p3, t.p1)));
    t.n1 = t.n2 = t.n3 = nn;
    t.mat = mid;
    t.src = offset + i;
  }
  if (range) { range[0] = offset; range[1] = (int32_t)s->tris.size(); }
  return RTS_OK;
}

int rts_scene_build_bvh(rts_scene* s, int leaf_size) {
  if (!s || leaf_size < 1) return RTS_ERR_ARG;
  if (s->built) return RTS_ERR_STATE;
  // dummy node 0 (src/core/Scene.h:189-195); its uninitialised index is encoded as 0
  Node dummy;
  dummy.left = 255; dummy.right = 128; dummy.n = 30; dummy.index = 0;
  dummy.AA = mk(1, 1, 0); dummy.BB = mk(0, 1, 0);
  s->nodes.clear();
  s->nodes.push_back(dummy);
  if (!s->tris.empty()) {
    const char* lit = getenv("RTS_BVH_LITERAL");  // the line-by-line restatement (checks the fast build)
    if (lit && atoi(lit)) build_sah(s->tris, s->nodes, 0, (int)s->tris.size() - 1, leaf_size);
    else build_sah_fast(s->tris, s->nodes, leaf_size);
  }
  s->built = true;
  return RTS_OK;
}

int rts_scene_counts(const rts_scene* s, int32_t* n_triangles, int32_t* n_nodes, int32_t* max_depth, int32_t* n_leaves) {
  if (!s) return RTS_ERR_ARG;
  if (n_triangles) *n_triangles = (int32_t)s->tris.size();
  if (n_nodes) *n_nodes = (int32_t)s->nodes.size();
  int32_t d = 0, l = 0;
  if (s->built) tree_stats(s->nodes, 1, d, l);
  if (max_depth) *max_depth = d;
  if (n_leaves) *n_leaves = l;
  return RTS_OK;
}

int rts_scene_encode(const rts_scene* s, float* tri_enc, float* node_enc) {
  if (!s) return RTS_ERR_ARG;
  if (tri_enc) {
    for (size_t i = 0; i < s->tris.size(); i++) {
      const Tri& t = s->tris[i];
      const rts_material& m = s->mats[t.mat];
      float* o = tri_enc + 42 * i;
      const v3 vs[6] = {t.p1, t.p2, t.p3, t.n1, t.n2, t.n3};
      for (int k = 0; k < 6; k++) { o[3 * k] = vs[k].x; o[3 * k + 1] = vs[k].y; o[3 * k + 2] = vs[k].z; }
      const float rest[24] = {m.emissive[0], m.emissive[1], m.emissive[2], m.base_color[0], m.base_color[1],
                              m.base_color[2], m.subsurface, m.metallic, m.specular, m.specular_tint, m.roughness,
                              m.anisotropic, m.sheen, m.sheen_tint, m.clearcoat, m.clearcoat_gloss, m.ior,
                              m.transmission, m.medium_color[0], m.medium_color[1], m.medium_color[2],
                              m.medium_type, m.medium_density, m.medium_anisotropy};
      memcpy(o + 18, rest, sizeof(rest));
    }
  }
  if (node_enc) {
    if (!s->built) return RTS_ERR_STATE;
    for (size_t i = 0; i < s->nodes.size(); i++) {
      const Node& n = s->nodes[i];
      float* o = node_enc + 12 * i;
      o[0] = (float)n.left; o[1] = (float)n.right; o[2] = 0;
      o[3] = (float)n.n; o[4] = (float)n.index; o[5] = 0;
      o[6] = n.AA.x; o[7] = n.AA.y; o[8] = n.AA.z;
      o[9] = n.BB.x; o[10] = n.BB.y; o[11] = n.BB.z;
    }
  }
  return RTS_OK;
}

int rts_scene_nodes(const rts_scene* s, int32_t* left, int32_t* right, int32_t* n, int32_t* index, float* aa, float* bb) {
  if (!s || !s->built) return RTS_ERR_STATE;
  for (size_t i = 0; i < s->nodes.size(); i++) {
    const Node& nd = s->nodes[i];
    if (left) left[i] = nd.left;
    if (right) right[i] = nd.right;
    if (n) n[i] = nd.n;
    if (index) index[i] = nd.index;
    if (aa) { aa[3 * i] = nd.AA.x; aa[3 * i + 1] = nd.AA.y; aa[3 * i + 2] = nd.AA.z; }
    if (bb) { bb[3 * i] = nd.BB.x; bb[3 * i + 1] = nd.BB.y; bb[3 * i + 2] = nd.BB.z; }
  }
  return RTS_OK;
}

int rts_scene_export_soa(const rts_scene* s, float* p1, float* p2, float* p3, float* n1, float* n2, float* n3,
                         int32_t* material_id, rts_material* materials, int32_t* n_materials) {
  if (!s) return RTS_ERR_ARG;
  // compact the material list to the materials still referenced, in first-use order
  std::vector<int> remap(s->mats.size(), -1);
  std::vector<rts_material> used;
  for (const Tri& t : s->tris) {
    if (remap[t.mat] < 0) {
      int found = -1;
      for (size_t k = 0; k < used.size(); k++)
        if (same_material(used[k], s->mats[t.mat])) { found = (int)k; break; }
      if (found < 0) { used.push_back(s->mats[t.mat]); found = (int)used.size() - 1; }
      remap[t.mat] = found;
    }
  }
  if (n_materials) *n_materials = (int32_t)used.size();
  if (materials) memcpy(materials, used.data(), used.size() * sizeof(rts_material));
  for (size_t i = 0; i < s->tris.size(); i++) {
    const Tri& t = s->tris[i];
    float* outs[6] = {p1, p2, p3, n1, n2, n3};
    const v3 vs[6] = {t.p1, t.p2, t.p3, t.n1, t.n2, t.n3};
    for (int k = 0; k < 6; k++)
      if (outs[k]) { outs[k][3 * i] = vs[k].x; outs[k][3 * i + 1] = vs[k].y; outs[k][3 * i + 2] = vs[k].z; }
    if (material_id) material_id[i] = remap[t.mat];
  }
  return RTS_OK;
}

int rts_scene_set_material(rts_scene* s, int first, int count, const rts_material* mat) {
  if (!s || !mat || first < 0 || count < 0 || (size_t)first + (size_t)count > s->tris.size()) return RTS_ERR_ARG;
  int mid = add_material(s, *mat);
  for (int i = first; i < first + count; i++) s->tris[i].mat = mid;
  return RTS_OK;
}

int rts_scene_post_bvh_index(const rts_scene* s, int32_t* pre_to_post) {
  if (!s || !pre_to_post) return RTS_ERR_ARG;
  for (size_t i = 0; i < s->tris.size(); i++) pre_to_post[s->tris[i].src] = (int32_t)i;
  return RTS_OK;
}

// ------------------------------------------------------------------------- HDR decode
// Restates thirdparty/hdrloader/hdrloader.cpp:29-190 over an in-memory file.
namespace {
struct Reader {
  const unsigned char* d;
  size_t n, pos;
  bool eof;
  int getc() {
    if (pos >= n) { eof = true; return -1; }
    return d[pos++];
  }
};
static bool old_decrunch(unsigned char (*scan)[4], int len, Reader& f) {  // HDRL:161-190
  int rshift = 0;
  while (len > 0) {
    scan[0][0] = (unsigned char)f.getc();
    scan[0][1] = (unsigned char)f.getc();
    scan[0][2] = (unsigned char)f.getc();
    scan[0][3] = (unsigned char)f.getc();
    if (f.eof) return false;
    if (scan[0][0] == 1 && scan[0][1] == 1 && scan[0][2] == 1) {
      for (int i = scan[0][3] << rshift; i > 0; i--) {
        memcpy(&scan[0][0], &scan[-1][0], 4);
        scan++;
        len--;
      }
      rshift += 8;
    } else {
      scan++;
      len--;
      rshift = 0;
    }
  }
  return true;
}
static bool decrunch(unsigned char (*scan)[4], int len, Reader& f) {  // HDRL:118-159
  if (len < 8 || len > 0x7fff) return old_decrunch(scan, len, f);
  int i = f.getc();
  if (i != 2) {
    if (i >= 0) f.pos--;
    return old_decrunch(scan, len, f);
  }
  scan[0][1] = (unsigned char)f.getc();
  scan[0][2] = (unsigned char)f.getc();
  i = f.getc();
  if (scan[0][1] != 2 || (scan[0][2] & 128)) {
    scan[0][0] = 2;
    scan[0][3] = (unsigned char)i;
    return old_decrunch(scan + 1, len - 1, f);
  }
  for (i = 0; i < 4; i++) {
    for (int j = 0; j < len;) {
      unsigned char code = (unsigned char)f.getc();
      if (code > 128) {
        code &= 127;
        unsigned char val = (unsigned char)f.getc();
        while (code-- && j < len) scan[j++][i] = val;
      } else {
        while (code-- && j < len) scan[j++][i] = (unsigned char)f.getc();
      }
      if (f.eof) return false;
    }
  }
  return !f.eof;
}
static float convert_component(int expo, int val) {  // HDRL:99-104
  float v = (float)val / 256.0f;
  float d = (float)pow(2.0, (double)expo);
  return v * d;
}
}  // namespace

int rts_hdr_load(const char* path, int32_t* width, int32_t* height, float** out_rgb) {
  if (!path || !width || !height || !out_rgb) return RTS_ERR_ARG;
  *out_rgb = nullptr;
  FILE* fp = fopen(path, "rb");
  if (!fp) return RTS_ERR_IO;
  std::vector<unsigned char> data;
  unsigned char buf[1 << 16];
  size_t k;
  while ((k = fread(buf, 1, sizeof(buf), fp)) > 0) data.insert(data.end(), buf, buf + k);
  fclose(fp);
  Reader f{data.data(), data.size(), 0, false};
  if (data.size() < 11 || memcmp(data.data(), "#?RADIANCE", 10) != 0) return RTS_ERR_FORMAT;
  f.pos = 11;  // fread(10) + fseek(1)
  int c = 0, oldc;
  while (true) {  // header ends at an empty line
    oldc = c;
    c = f.getc();
    if (c < 0) return RTS_ERR_FORMAT;
    if (c == 0xa && oldc == 0xa) break;
  }
  std::string reso;
  while (true) {
    c = f.getc();
    if (c < 0) return RTS_ERR_FORMAT;
    reso.push_back((char)c);
    if (c == 0xa) break;
  }
  int w = 0, h = 0;
  if (sscanf(reso.c_str(), "-Y %d +X %d", &h, &w) != 2 || w <= 0 || h <= 0) return RTS_ERR_FORMAT;  // R15 fixed
  float* cols = (float*)malloc(sizeof(float) * 3 * (size_t)w * h);
  if (!cols) return RTS_ERR_NOMEM;
  memset(cols, 0, sizeof(float) * 3 * (size_t)w * h);
  std::vector<unsigned char> scanline(4 * (size_t)(w + 1));
  unsigned char(*scan)[4] = reinterpret_cast<unsigned char(*)[4]>(scanline.data() + 4);  // scan[-1] valid
  float* out = cols;
  for (int y = h - 1; y >= 0; y--) {
    if (!decrunch(scan, w, f)) break;
    for (int x = 0; x < w; x++) {  // workOnRGBE HDRL:106-116
      int expo = scan[x][3] - 128;
      out[0] = convert_component(expo, scan[x][0]);
      out[1] = convert_component(expo, scan[x][1]);
      out[2] = convert_component(expo, scan[x][2]);
      out += 3;
    }
  }
  *width = w;
  *height = h;
  *out_rgb = cols;
  return RTS_OK;
}

void rts_free(void* p) { free(p); }

// calculateHdrCache (src/core/Utility.h:33-131), literal evaluation order.
int rts_hdr_cache(const float* HDR, int width, int height, float* cache) {
  if (!HDR || !cache || width <= 0 || height <= 0) return RTS_ERR_ARG;
  size_t W = (size_t)width, Hh = (size_t)height;
  float lumSum = 0.0f;
  std::vector<float> pdf(W * Hh);
  for (size_t i = 0; i < Hh; i++)
    for (size_t j = 0; j < W; j++) {
      float R = HDR[3 * (i * W + j)], G = HDR[3 * (i * W + j) + 1], B = HDR[3 * (i * W + j) + 2];
      float lum = (float)(0.2 * (double)R + 0.7 * (double)G + 0.1 * (double)B);
      pdf[i * W + j] = lum;
      lumSum += lum;
    }
  for (size_t i = 0; i < Hh; i++)
    for (size_t j = 0; j < W; j++) pdf[i * W + j] /= lumSum;
  std::vector<float> pdf_x_margin(W, 0.0f);
  for (size_t j = 0; j < W; j++)
    for (size_t i = 0; i < Hh; i++) pdf_x_margin[j] += pdf[i * W + j];
  std::vector<float> cdf_x_margin = pdf_x_margin;
  for (size_t i = 1; i < W; i++) cdf_x_margin[i] += cdf_x_margin[i - 1];
  // conditional cdf of y given x, stored column-major: cdf_y[j][i]
  std::vector<float> cdf_y(W * Hh);
  for (size_t j = 0; j < W; j++) {
    float acc = 0.0f;
    for (size_t i = 0; i < Hh; i++) {
      float pc = pdf[i * W + j] / pdf_x_margin[j];
      acc = (i == 0) ? pc : acc + pc;
      cdf_y[j * Hh + i] = acc;
    }
  }
  for (size_t j = 0; j < W; j++)
    for (size_t i = 0; i < Hh; i++) {
      float xi_1 = (float)i / (float)height;
      float xi_2 = (float)j / (float)width;
      size_t x = (size_t)(std::lower_bound(cdf_x_margin.begin(), cdf_x_margin.end(), xi_1) - cdf_x_margin.begin());
      if (x >= W) x = W - 1;  // the reference reads out of bounds here; never reached on valid maps
      const float* col = &cdf_y[x * Hh];
      size_t y = (size_t)(std::lower_bound(col, col + Hh, xi_2) - col);
      float* o = cache + 3 * (i * W + j);
      o[0] = (float)x / (float)width;
      o[1] = (float)y / (float)height;
      o[2] = pdf[i * W + j];
    }
  return RTS_OK;
}

// Camera::updateCameraVectors (src/core/Camera.h:160-174) with WorldUp = (0,1,0).
int rts_camera(float yaw_deg, float pitch_deg, float zoom_deg, float screen_ratio, float* out) {
  if (!out) return RTS_ERR_ARG;
  v3 front = mk(cosf(radians(yaw_deg)) * cosf(radians(pitch_deg)), sinf(radians(pitch_deg)),
                sinf(radians(yaw_deg)) * cosf(radians(pitch_deg)));
  v3 Front = normalize3(front);
  v3 Right = normalize3(cross3(Front, mk(0, 1, 0)));
  v3 Up = normalize3(cross3(Right, Front));
  float halfH = tanf(radians(zoom_deg));
  float halfW = halfH * screen_ratio;
  v3 lbc = sub(sub(Front, mul(Right, halfW)), mul(Up, halfH));
  const v3 vs[4] = {Front, Right, Up, lbc};
  for (int k = 0; k < 4; k++) { out[3 * k] = vs[k].x; out[3 * k + 1] = vs[k].y; out[3 * k + 2] = vs[k].z; }
  out[12] = halfH;
  out[13] = halfW;
  out[14] = out[15] = out[16] = 0.0f;
  return RTS_OK;
}

// ------------------------------------------------------------------------------ PNG
// (static, distinct names: inside extern "C" a helper called crc32 would be the global C symbol
// and bind to zlib's crc32 in processes that load zlib)
static uint32_t png_crc_table[256];
static bool png_crc_ready = false;
static uint32_t png_crc32(const unsigned char* d, size_t n, uint32_t c = 0xffffffffu) {
  if (!png_crc_ready) {
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t v = i;
      for (int k = 0; k < 8; k++) v = (v & 1u) ? 0xedb88320u ^ (v >> 1) : v >> 1;
      png_crc_table[i] = v;
    }
    png_crc_ready = true;
  }
  for (size_t i = 0; i < n; i++) c = png_crc_table[(c ^ d[i]) & 0xffu] ^ (c >> 8);
  return c;
}
static void png_put32(std::vector<unsigned char>& v, uint32_t x) {
  v.push_back((unsigned char)(x >> 24)); v.push_back((unsigned char)(x >> 16));
  v.push_back((unsigned char)(x >> 8)); v.push_back((unsigned char)x);
}
static void png_chunk(FILE* f, const char* type, const std::vector<unsigned char>& data) {
  std::vector<unsigned char> b;
  png_put32(b, (uint32_t)data.size());
  b.insert(b.end(), type, type + 4);
  b.insert(b.end(), data.begin(), data.end());
  const uint32_t c = png_crc32(b.data() + 4, b.size() - 4) ^ 0xffffffffu;
  png_put32(b, c);
  fwrite(b.data(), 1, b.size(), f);
}
int rts_write_png(const char* path, int width, int height, const uint8_t* rgb) {
  if (!path || !rgb || width <= 0 || height <= 0) return RTS_ERR_ARG;
  FILE* f = fopen(path, "wb");
  if (!f) return RTS_ERR_IO;
  static const unsigned char sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  fwrite(sig, 1, 8, f);
  std::vector<unsigned char> ihdr;
  png_put32(ihdr, (uint32_t)width);
  png_put32(ihdr, (uint32_t)height);
  const unsigned char rest[5] = {8, 2, 0, 0, 0};  // 8-bit, RGB, deflate, filter 0, no interlace
  ihdr.insert(ihdr.end(), rest, rest + 5);
  png_chunk(f, "IHDR", ihdr);
  // zlib stream of stored deflate blocks over the filtered scanlines (filter byte 0)
  const size_t row = (size_t)width * 3 + 1, raw = row * (size_t)height;
  std::vector<unsigned char> z;
  z.reserve(raw + raw / 65535 * 5 + 16);
  z.push_back(0x78);
  z.push_back(0x01);
  uint32_t s1 = 1, s2 = 0;  // Adler-32
  size_t pos = 0;
  std::vector<unsigned char> block;
  while (pos < raw) {
    const size_t n = std::min<size_t>(65535, raw - pos);
    z.push_back(pos + n == raw ? 1 : 0);
    z.push_back((unsigned char)(n & 0xff)); z.push_back((unsigned char)(n >> 8));
    z.push_back((unsigned char)(~n & 0xff)); z.push_back((unsigned char)((~n >> 8) & 0xff));
    for (size_t k = pos; k < pos + n; k++) {
      const size_t y = k / row, x = k % row;
      const unsigned char b = x == 0 ? 0 : rgb[y * (size_t)width * 3 + (x - 1)];
      z.push_back(b);
      s1 = (s1 + b) % 65521u;
      s2 = (s2 + s1) % 65521u;
    }
    pos += n;
  }
  png_put32(z, (s2 << 16) | s1);
  png_chunk(f, "IDAT", z);
  png_chunk(f, "IEND", std::vector<unsigned char>());
  const bool ok = fflush(f) == 0;
  fclose(f);
  return ok ? RTS_OK : RTS_ERR_IO;
}

// glibc rand() restated (stdlib/random_r.c, TYPE_3: x^31 + x^3 + 1 additive feedback over 31
// words, the default state of srand/rand), so the randOrigin list does not depend on the libc
// of the machine it runs on and has no length limit:
//   r[0] = seed (0 -> 1); r[i] = 16807 * r[i-1] mod (2^31 - 1), i = 1..30 (Schrage's form, as
//   glibc's __srandom_r); then r[i] = r[i-31] + r[i-3] (mod 2^32) for i >= 31, the first 310
//   outputs discarded (10 * 31), and rand() = r[i] >> 1 (RAND_MAX = 2^31 - 1).
int rts_glibc_rand(unsigned int seed, int n, int* out) {
  if (!out || n < 0) return RTS_ERR_ARG;
  uint32_t r[34];
  int32_t word = seed == 0 ? 1 : (int32_t)seed;
  r[0] = (uint32_t)word;
  for (int i = 1; i < 31; i++) {
    const int32_t hi = word / 127773, lo = word % 127773;
    word = 16807 * lo - 2836 * hi;
    if (word < 0) word += 2147483647;
    r[i] = (uint32_t)word;
  }
  // ring of the last 31 words: front = i - 31, rear = i - 3
  uint32_t ring[31];
  for (int i = 0; i < 31; i++) ring[i] = r[i];
  int f = 3, b = 0;  // glibc: fptr = state + SEP_3 (3), rptr = state
  auto next = [&]() -> uint32_t {
    ring[f] += ring[b];
    const uint32_t v = ring[f];
    if (++f == 31) f = 0;
    if (++b == 31) b = 0;
    return v >> 1;
  };
  for (int i = 0; i < 310; i++) (void)next();
  for (int k = 0; k < n; k++) out[k] = (int)next();
  return RTS_OK;
}

int rts_cpu_rand_origins(unsigned int seed, int n, float* out) {
  if (!out || n < 0) return RTS_ERR_ARG;
  std::vector<int> r((size_t)n);
  if (n > 0) rts_glibc_rand(seed, n, r.data());
  for (int k = 0; k < n; k++) {
    float x = (float)((float)r[k] / (2147483647 + 1.0));  // GetCPURandom, src/core/Utility.h:15-17
    out[k] = 674764.0f * (x + 1.0f);                      // main.cpp:190
  }
  return RTS_OK;
}

}  // extern "C"

int rts_tri_filter(const float* tri, int n_triangles, float* out, double* k, int32_t* flagged) {
  if (n_triangles < 0 || (n_triangles && (!tri || !out)) || !k) return RTS_ERR_ARG;
  const trif::Consts c = trif::build(tri, n_triangles, out);
  k[0] = c.k1;
  k[1] = c.k0;
  if (flagged) *flagged = c.flagged;
  return 0;
}
