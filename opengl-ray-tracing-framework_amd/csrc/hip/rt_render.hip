// rt_render.hip — librtamd.so: the C-ABI of include/rt_abi.h over the gfx950 path-tracing
// kernels of rt_kernels.h.  Host code here converts the reference's scene description
// (SoA or the reference's own AoS encodings) into the device layout, owns the device
// buffers and launches the persistent kernel.  No fallback path: without a HIP device every
// entry point returns RT_ERR_NODEVICE / RT_ERR_HIP.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <functional>
#include <new>
#include <string>
#include <vector>
#include <limits>

#include "rt_abi.h"
#include "rt_kernels.h"
#include "rt_wavefront.h"

#ifndef RT_SPLIT_KINDS  // bulk groups trace shadow rays and continuations in launches of their own (round 6)
#define RT_SPLIT_KINDS 1
#endif
#ifndef RT_SPLIT_PASSES  // the last pass traced split (later ones: one launch, both kinds); C3 3 / 4 / 5 / 6 / 7 vs 8:
                         // -0.18, -0.15 / +0.19, +0.22 / -0.03 / -0.04% (profiles/r06_ab_split_passes_C3.log)
#define RT_SPLIT_PASSES 5
#endif
#ifndef RT_SPLIT_CONT_FIRST  // split queues: the continuations' launch first (1) or the shadow rays' (0)
#define RT_SPLIT_CONT_FIRST 0  // C3 1 vs 0: -0.16% (profiles/r06_ab_split_knobs_C3.log)
#endif
#include "tri_filter.h"

using rtd::GNode;
using rtd::KParams;

struct rt_ctx {
  int device = 0;
  int n_cus = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  std::string err;
  // scene
  GNode* d_nodes = nullptr;
  rtd::QNode* d_qnodes = nullptr;
  int qroot = 0, qstack_entries = 2, n_qnodes = 0;
  bool wide = false;                          // 4-wide traversal available for this scene
  float4* d_tri = nullptr;
  float4* d_trx = nullptr;  // traversal records (tri_filter.h)
  double tri_k1 = 0.0, tri_k0 = 0.0;  // their edge-filter margin
  int tri_flagged = 0;
  float4* d_trin = nullptr;
  float4* d_hrec = nullptr;  // the shade's hit records (KParams::hrec)
  float4* d_mats = nullptr;
  int n_tri = 0, n_mats = 0, root = 0, has_scene = 0, stack_entries = 2;
  double cull_R = 0.0, cull_K = 0.0, cull_off = 0.0;  // culling bound of the scene (cull_bound_stats)
  bool scene_set = false;
  std::vector<int32_t> tri_mat;  // host copy of the per-triangle material ids (for updates)
  std::vector<float> mat_table;  // host copy, 32 floats per material
  // env
  float4* d_hdr = nullptr;
  float2* d_cache = nullptr;                  // hdrCache.rg; d_hdr = {hdrMap.rgb, hdrCache.b}
  // NEE light samples per hdrCache texel (rt_light_table_kernel) for one envAngle each: two tables,
  // so a call whose angle differs from the previous call's rebuilds the other table on its own
  // stream after the last call that read that one (an event), without draining calls in flight
  struct LightTable {
    float4* d = nullptr;
    bool valid = false;
    float angle = 0.0f;                       // the envAngle d was built for
    hipEvent_t last_use = nullptr;            // on the ctx stream after the last call that read d
    hipEvent_t built = nullptr;               // after the kernel that last built d (on that call's stream)
  };
  LightTable light[2];
  int light_cur = 0;                          // the table the last call used
  int hdr_w = 0, hdr_h = 0, hdr_res = 0;
  bool env_set = false;
  // frame
  int W = 0, H = 0, tile_w = 32, tile_h = 32, tiles_x = 0, tiles_y = 0, rank = 0, world = 1;
  int local_tiles = 0, max_local_tiles = 0;
  float4* d_accum = nullptr;
  bool frame_set = false;
  int loop_num = 0;
  // counters
  unsigned int* d_counter = nullptr;
  unsigned long long* d_stats = nullptr;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> events;        // whole render calls
  struct TraceEv {
    hipEvent_t s, e;
    uint64_t call;  // the render call (its index in `launches`) that queued the launch
  };
  std::vector<TraceEv> trace_events;  // traversal launches
  std::vector<hipEvent_t> event_pool;
  double kernel_ms = 0.0, trace_ms = 0.0;
  // Union of the traversal launches' intervals (rt_stats.trace_busy_ms).  Each folded launch is
  // placed on a double-precision timeline by its start's offset from the previously folded
  // launch's start (busy_anchor, at busy_anchor_t ms), so an offset is a short float interval
  // however long the context lives.  Intervals that can no longer overlap a pending launch are
  // summed into busy_closed_ms and dropped: a launch of call k starts after every launch of
  // call k-2 has ended (pipelined calls wait for their set's previous call; the ctx stream joins
  // each call's streams), so folding call k's launches closes the intervals of calls <= k-2 and
  // the open list holds about two calls' worth.
  struct BusyIv {
    double lo, hi;
    uint64_t call;  // the newest call merged into the interval
  };
  hipEvent_t busy_anchor = nullptr;
  double busy_anchor_t = 0.0;
  std::vector<BusyIv> busy;
  double busy_closed_ms = 0.0;
  uint64_t launches = 0, trace_launches = 0;
  int blocks_per_cu = 0, block_lds = 0;      // megakernel
  int trace_bpc = 0, trace_bpc0 = 0;          // wavefront traversal blocks/CU (passes >= 1, pass 0)
  int trace_lds_entries = 0, trace_lds = 0;
  int split_kinds = RT_SPLIT_KINDS;  // bulk groups: shadow rays and continuations in queues of their own
  int split_passes = RT_SPLIT_PASSES;  // ... in passes 1 .. split_passes (later ones: one queue, one launch)
  // per-frame loopNum / randOrigin of one render call: pinned host staging -> device table;
  // ft[0] for batched calls, ft[1 + p] for pipelined one-frame calls on pipeline set p
  struct FrameTable {
    int* h = nullptr;                         // [cap] loop_num then [cap] rand_origin bits
    int* d = nullptr;                         // + [cap][4] float2 Sobol pairs (wf_sobol)
    size_t cap = 0;
    hipEvent_t ev = nullptr;                  // the last upload (the host table is reused after it)
  };
  FrameTable ft[5];
#ifndef RT_CAM_SHADE  // the bulk camera pass's shade in its own instantiation (wf_shade<..., CAM>)
#define RT_CAM_SHADE 1
#endif
#ifndef RT_POOL_CHUNK_DEFAULT
#define RT_POOL_CHUNK_DEFAULT 1024
#endif
  int pool_chunk = RT_POOL_CHUNK_DEFAULT;     // rays per queue atomic in wf_trace (C3: 256 -> 512 -> 1024: +2.3%, +2.4%)
  int2* d_stack_ovf = nullptr;
  void* d_disp = nullptr;                     // rt_tonemap output (W*H*3 bytes)
  size_t disp_bytes = 0;
  void* d_gather = nullptr;                   // rt_gather on rank 0: every rank's tiles, then the frame
  // rt_gather over RCCL: the communicators (one per rank, this process drives them all) of the
  // device set ctxs[0] last gathered over, and the transport its last gather used
  std::vector<int> rccl_devs;
  std::vector<ncclComm_t> rccl_comms;
  int gather_transport = 0;
  size_t gather_bytes = 0;
  size_t stack_ovf_bytes = 0;
  // wavefront path state (one slot per local pixel)
  void* wf_mem = nullptr;
  size_t wf_paths = 0;                        // path slots per frame group
  rtd::WFState wf{};                          // pixel lists (shared by every group)
  // Frame groups: the frames of one batch are split into n_groups independent wavefronts with
  // their own path state, run on their own streams, so the latency tail of one group's late
  // bounces overlaps the other's busy passes; blends stay in frame order (events).
  static constexpr int MAX_GROUPS = 4;
  int n_groups = 2;
  // rt_order_work's costly head: the first order_head work items (whole 64-item blocks) are the
  // costliest blocks and form pixel group 0 of a one-frame call; 0 = even split
  size_t order_head = 0;
  rtd::WFState wfg[MAX_GROUPS]{};
  hipStream_t aux[MAX_GROUPS] = {};
  unsigned int* d_pix = nullptr;   // pixel list of this rank: xy then accumulation index
  // tile ownership: owner[t] = rank of global tile t (default t % world; rt_set_tile_owners);
  // my_tiles = this rank's global tiles in local order; tile_src[t] = (rank, local index)
  std::vector<int32_t> owner, my_tiles;
  int* d_tile_ids = nullptr;       // my_tiles on the device (KParams.tile_ids)
  int2* d_tile_src = nullptr;      // tile_src on the device (rt_assemble_kernel)
  unsigned long long* d_tile_cost = nullptr;  // rt_tile_costs: per local tile, during the probe only
  bool tile_cost_on = false;
  bool cost_blocks = false;        // the probe counts per 64-item work block (rt_order_work)
  float4* d_cam = nullptr;         // per pixel of this rank: camera direction, u * v (wf_camera), then the
                                   // per-pixel camera hit points (WFState::org), one of each per set
  int cam_sets = 1;                // camera tables in d_cam (one per pipeline set, n_valid each)
  int n_valid = 0;                 // valid pixels of this rank (work items of the wavefront)
  int frames_cap = 1;              // frames in flight per wavefront
  size_t max_slots_req = 0;        // rt_set_max_paths (0: RT_MAX_SLOTS or the 320 Mi default)
  // path-persistent finisher (wf_finish): a frame group of at most finish_slots path slots runs
  // passes 0 .. finish_pass-1 as wavefront passes, then one wf_finish launch ends every path
  int finish_pass = 2;  // C3 1080p single frames: 1 / 2 / 3 -> 3.73 / 3.35 / 3.41 ms (off: 3.79)
  uint64_t finish_slots = uint64_t(8) << 20;
  int finish_bpc = 0;              // wf_finish blocks per CU
  // Pipelined one-frame calls (rt_set_pipeline, depth D = 2): one-frame call k runs as a single
  // group on stream aux[1 + p], p = k mod D, with path-state set wfg[p], camera table p and frame
  // table ft[1 + p], so call k+1's early passes fill the CUs that call k's latency-bound finisher
  // leaves idle.  Only the blend waits for the caller's stream (history, frame order); the caller's
  // stream still joins each call at its end.  set_free[p]: the last call on set p has finished;
  // batch_done: the last batched (non-pipelined) call has finished.
  // rt_tonemap_async: display passes read back into pinned host slots, fetched later
  static constexpr int DISP_SLOTS = 4;
  struct DisplaySlot {
    uint8_t* host = nullptr;
    size_t cap = 0, bytes = 0;
    hipEvent_t ev = nullptr;
  };
  DisplaySlot disp[DISP_SLOTS];
  int pipe_depth = 1;
  int pipe_next = 0;
  size_t pipe_nomem_slots = SIZE_MAX;  // pipelined batches this large did not fit twice
  // a pipelined call's finisher runs 2 of its 3 resident blocks per CU, leaving room for the next
  // call's passes: C3 1080p back-to-back 2.33 -> 2.10 ms (1 block: the same; synchronised 3.33 ->
  // 3.24 ms, 1 block 3.50)
  int pipe_finish_bpc = 2;
  int pipe_finish_pass = -1;  // -1: finish_pass
  hipEvent_t set_free[MAX_GROUPS] = {};
  hipEvent_t batch_done = nullptr;
};

namespace {

// Development settings (measurement and test builds only).  The release library honours only the
// C-ABI (include/rt_abi.h); `make` also builds lib/librtamd_dev.so with -DRT_DEV, where these
// environment variables reach the code they name: the test-only culling switch of
// tests/test_gpu_cull.py (RT_CULL_EPS_SCALE), the traversal-structure variants the parity tests
// cover (RT_BVH_WIDTH, RT_REBUILD, RT_COLLAPSE, RT_QBFS) and the occupancy / grouping / finisher
// parameters the A/B tools sweep.
inline const char* knob(const char* name) {
#ifdef RT_DEV
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

int fail(rt_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}
#define HIPCHK(ctx, call)                                                                        \
  do {                                                                                           \
    hipError_t e_ = (call);                                                                      \
    if (e_ != hipSuccess)                                                                        \
      return fail((ctx), RT_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_));         \
  } while (0)

template <typename T>
void dfree(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

// Same fp32 operations as the shader's per-test N = normalize(cross(p2-p1, p3-p1)) (RT:253).
inline void geometric_normal(const float* p1, const float* p2, const float* p3, float* n) {
  float ax = p2[0] - p1[0], ay = p2[1] - p1[1], az = p2[2] - p1[2];
  float bx = p3[0] - p1[0], by = p3[1] - p1[1], bz = p3[2] - p1[2];
  float cx = ay * bz - by * az, cy = az * bx - bz * ax, cz = ax * by - bx * ay;
  float inv = 1.0f / sqrtf(cx * cx + cy * cy + cz * cz);
  n[0] = cx * inv; n[1] = cy * inv; n[2] = cz * inv;
}

// Culling bound ("What the culling margin covers").  A subtree may be skipped when
// its box entry t0 exceeds the best hit; that is exact only if no triangle inside the box can be
// accepted by the reference's test (RT:241-299) at a computed t below t0.  An accepted hit point
// P = S + d*t (fp32) lies within eps (per axis) of its triangle, hence of every box holding it:
//   off-plane |(P - p1).N| <= 36 u R  (rounding of RT:265 and of P; R bounds |coords|, origins),
//   in-plane slack of the three edge signs <= 70 u R / cos(theta)  (theta: fp32 N vs exact normal),
//   X = S + d*t (exact) vs P: <= 8 u R,
//   + the triangle's vertices off the plane (p1, N): max_k |(pk - p1).N|,
// so t >= t0 - eps * max|1/d_a|.  Returned per scene: K (units of u R) and off; the render
// doubles eps = K u R + off as safety.  Degenerate (zero-area with a finite fp32 normal) or badly
// conditioned triangles, or triangles outside their leaf box, give K = inf: no culling.
struct CullStats {
  double R = 0.0, K = 0.0, off = 0.0;
};
CullStats cull_bound_stats(const rt_scene_soa* s) {
  CullStats cs;
  const int nt = s->n_triangles;
  for (int i = 0; i < nt; i++) {
    const float* p[3] = {s->p1 + 3 * i, s->p2 + 3 * i, s->p3 + 3 * i};
    float ng[3];
    geometric_normal(p[0], p[1], p[2], ng);
    for (int k = 0; k < 3; k++)
      for (int a = 0; a < 3; a++) cs.R = std::max(cs.R, std::fabs((double)p[k][a]));
    if (!(std::isfinite(ng[0]) && std::isfinite(ng[1]) && std::isfinite(ng[2]))) continue;  // never hit (NaN tests)
    double e1[3], e2[3], cx[3];
    for (int a = 0; a < 3; a++) { e1[a] = (double)p[1][a] - p[0][a]; e2[a] = (double)p[2][a] - p[0][a]; }
    cx[0] = e1[1] * e2[2] - e1[2] * e2[1];
    cx[1] = e1[2] * e2[0] - e1[0] * e2[2];
    cx[2] = e1[0] * e2[1] - e1[1] * e2[0];
    const double nrm = std::sqrt(cx[0] * cx[0] + cx[1] * cx[1] + cx[2] * cx[2]);
    const double cosT = nrm > 0.0 ? (ng[0] * cx[0] + ng[1] * cx[1] + ng[2] * cx[2]) / nrm : 0.0;
    if (!(cosT > 0.25)) { cs.K = INFINITY; continue; }
    cs.K = std::max(cs.K, 44.0 + 70.0 / cosT);
    for (int k = 1; k < 3; k++) {
      double o = 0.0;
      for (int a = 0; a < 3; a++) o += ((double)p[k][a] - p[0][a]) * ng[a];
      cs.off = std::max(cs.off, std::fabs(o));
    }
  }
  // every leaf's triangles inside the leaf's box (the reference's own boxes are their min/max)
  for (int n = 1; n < s->n_nodes && s->node_n; n++) {
    if (s->node_n[n] <= 0) continue;
    for (int i = s->node_index[n]; i < s->node_index[n] + s->node_n[n] && i < nt; i++)
      for (const float* q : {s->p1 + 3 * i, s->p2 + 3 * i, s->p3 + 3 * i})
        for (int a = 0; a < 3; a++)
          if (!(q[a] >= s->node_aa[3 * n + a] && q[a] <= s->node_bb[3 * n + a])) cs.K = INFINITY;
  }
  return cs;
}

// Material.h fields -> 32-float device entry; ax/ay by getMaterial's formula (RT:205-207).
void pack_material(const rt_material& m, float* o) {
  const float* f = reinterpret_cast<const float*>(&m);
  for (int k = 0; k < 24; k++) o[k] = f[k];
  float aspect = gm::sqrt_(1.0f - m.anisotropic * 0.9f);
  o[24] = gm::max_(0.001f, (m.roughness * m.roughness) / aspect);
  o[25] = gm::max_(0.001f, (m.roughness * m.roughness) * aspect);
  int mt = (int)m.medium_type;
  memcpy(&o[26], &mt, 4);
  o[27] = o[28] = o[29] = o[30] = o[31] = 0.0f;
}

// New internal levels over the reference's leaves.  A leaf keeps its triangle range and its exact
// box (the reference's, RT:363-368); every internal box is the exact min/max union of the boxes
// below it.  The slab arithmetic is monotone in the box planes, so a box can only be hit when
// every box above it is: the traversal reaches exactly the leaves whose own box the reference's
// ray hits, whatever the internal levels are (the reference's exact-tie order is kept separately,
// by the leaf ranks of its own tree).  The reference's top levels are X-median splits (R18: SAH
// costs above INF = 114514 fall back to the median), so a full-sweep SAH over the leaf boxes
// (centroid order per axis, cost = area x triangles) gives a tree with fewer node visits.
// Returns the root of `out` (binary GNodes, host only: the device keeps the reference tree).
int rebuild_over_leaves(const std::vector<GNode>& gn, int root, std::vector<GNode>& out) {
  struct Box {
    float lo[3], hi[3];
  };
  struct Prim {
    int ref, n;
    Box b;
    double c[3];
  };
  auto is_leaf = [](int r) { return ((uint32_t)r & rtd::LEAF_BIT) != 0u; };
  std::vector<Prim> prims;
  std::vector<int> st{root};
  while (!st.empty()) {
    const GNode g = gn[st.back()];
    st.pop_back();
    const Box bl = {{g.b0.x, g.b0.y, g.b0.z}, {g.b0.w, g.b1.x, g.b1.y}};
    const Box br = {{g.b1.z, g.b1.w, g.b2.x}, {g.b2.y, g.b2.z, g.b2.w}};
    const int refs[2] = {g.ref.x, g.ref.y};
    const Box* boxes[2] = {&bl, &br};
    for (int k = 0; k < 2; k++) {
      if (!is_leaf(refs[k])) { st.push_back(refs[k]); continue; }
      Prim p;
      p.ref = refs[k];
      p.n = (int)((uint32_t)refs[k] & 15u) + 1;      p.b = *boxes[k];
      for (int a = 0; a < 3; a++) p.c[a] = 0.5 * ((double)p.b.lo[a] + (double)p.b.hi[a]);
      prims.push_back(p);
    }
  }
  auto unite = [](const Box& a, const Box& b) {
    Box u;
    for (int k = 0; k < 3; k++) { u.lo[k] = std::min(a.lo[k], b.lo[k]); u.hi[k] = std::max(a.hi[k], b.hi[k]); }
    return u;
  };
  auto area = [](const Box& b) {
    double e[3];
    for (int k = 0; k < 3; k++) e[k] = std::max(0.0, (double)b.hi[k] - (double)b.lo[k]);
    return e[0] * e[1] + e[1] * e[2] + e[2] * e[0];
  };
  std::vector<int> idx(prims.size()), tmp(prims.size());
  for (size_t i = 0; i < idx.size(); i++) idx[i] = (int)i;
  std::vector<double> right_cost(prims.size() + 1);
  out.clear();
  out.reserve(prims.size());
  std::function<int(int, int, Box&)> rec = [&](int b, int e, Box& box) -> int {
    if (e - b == 1) {
      box = prims[idx[b]].b;
      return prims[idx[b]].ref;
    }
    double best = 1e300;
    int bax = 0, bpos = b + (e - b) / 2;
    for (int ax = 0; ax < 3; ax++) {
      std::copy(idx.begin() + b, idx.begin() + e, tmp.begin() + b);
      std::sort(tmp.begin() + b, tmp.begin() + e, [&](int x, int y) {
        return prims[x].c[ax] < prims[y].c[ax] || (prims[x].c[ax] == prims[y].c[ax] && x < y);
      });
      Box acc = prims[tmp[e - 1]].b;
      int cnt = 0;
      for (int i = e - 1; i > b; i--) {  // right_cost[i] = cost of [i, e)
        acc = unite(acc, prims[tmp[i]].b);
        cnt += prims[tmp[i]].n;
        right_cost[i - b] = area(acc) * cnt;
      }
      acc = prims[tmp[b]].b;
      cnt = 0;
      for (int i = b; i < e - 1; i++) {  // split after i: [b, i] | [i + 1, e)
        acc = unite(acc, prims[tmp[i]].b);
        cnt += prims[tmp[i]].n;
        const double c = area(acc) * cnt + right_cost[i + 1 - b];
        if (c < best) { best = c; bax = ax; bpos = i + 1; }
      }
    }
    std::sort(idx.begin() + b, idx.begin() + e, [&](int x, int y) {
      return prims[x].c[bax] < prims[y].c[bax] || (prims[x].c[bax] == prims[y].c[bax] && x < y);
    });
    const int me = (int)out.size();
    out.push_back(GNode{});
    Box lb, rb;
    const int lr = rec(b, bpos, lb), rr = rec(bpos, e, rb);
    GNode g;
    memset(&g, 0, sizeof(g));
    g.b0 = make_float4(lb.lo[0], lb.lo[1], lb.lo[2], lb.hi[0]);
    g.b1 = make_float4(lb.hi[1], lb.hi[2], rb.lo[0], rb.lo[1]);
    g.b2 = make_float4(rb.lo[2], rb.hi[0], rb.hi[1], rb.hi[2]);
    g.ref = make_int4(lr, rr, 0, 0);
    out[me] = g;
    box = unite(lb, rb);
    return me;
  };
  Box rootbox;
  return rec(0, (int)prims.size(), rootbox);
}

// Leaf ranks + 4-wide collapse of the binary tree.
// * Leaf rank = position of the leaf in the reference's left-first DFS; gn[k].ref.z = rank of
//   the first leaf of node k's right subtree; trin[3t+1].w = rank of triangle t's leaf.  These
//   let the 4-wide traversal break exact distance ties the way the reference's visit order does.
// * A QNode replaces a binary node and a cut of its subtree with at most 4 slots, chosen by the
//   SAH-optimal collapse below (or greedily, largest area first).  Boxes are copied bit for bit.  A (grand)child box can only be hit when every box above it is
//   (children are min/max over subsets, and the slab arithmetic is monotone), so the 4-wide
//   traversal reaches exactly the reference's leaves.
// Returns false (binary traversal only) when a triangle belongs to two leaves.
bool build_wide(std::vector<GNode>& gn, int root, std::vector<float4>& trin, std::vector<rtd::QNode>& qn,
                int& qroot, int& qdepth) {
  const int nt = (int)(trin.size() / 3);
  auto is_leaf = [](int r) { return ((uint32_t)r & rtd::LEAF_BIT) != 0u; };
  auto first_of = [](int r) { return (int)(((uint32_t)r & 0x7fffffffu) >> 4); };
  auto count_of = [](int r) { return (int)((uint32_t)r & 15u) + 1; };
  std::vector<int> tri_rank(nt, -1);
  int rank = 0;
  bool ok = true;
  std::function<void(int)> rank_dfs = [&](int r) {
    if (is_leaf(r)) {
      for (int t = first_of(r); t < first_of(r) + count_of(r); t++) {
        if (tri_rank[t] >= 0) ok = false;
        tri_rank[t] = rank;
      }
      rank++;
      return;
    }
    rank_dfs(gn[r].ref.x);
    gn[r].ref.z = rank;
    rank_dfs(gn[r].ref.y);
  };
  rank_dfs(root);
  for (int t = 0; t < nt; t++) {
    float w;
    memcpy(&w, &tri_rank[t], 4);
    trin[3 * t + 1].w = w;
  }
  if (!ok) return false;
  // The tree that gets collapsed: by default internal levels rebuilt over the reference's leaves
  // (rebuild_over_leaves), RT_REBUILD=0 keeps the reference's own internal nodes.
  std::vector<GNode> rebuilt;
  int croot = root;
  const std::vector<GNode>* T = &gn;
  const char* re = knob("RT_REBUILD");
  if (!is_leaf(root) && !(re && atoi(re) == 0)) {
    croot = rebuild_over_leaves(gn, root, rebuilt);
    T = &rebuilt;
  }
  struct Slot {
    int ref;
    float lo[3], hi[3];
  };
  auto kids = [&](int b, Slot& L, Slot& R) {
    const GNode& g = (*T)[b];
    L = Slot{g.ref.x, {g.b0.x, g.b0.y, g.b0.z}, {g.b0.w, g.b1.x, g.b1.y}};
    R = Slot{g.ref.y, {g.b1.z, g.b1.w, g.b2.x}, {g.b2.y, g.b2.z, g.b2.w}};
  };
  auto area = [](const Slot& s) {
    double e[3];
    for (int k = 0; k < 3; k++) e[k] = (double)s.hi[k] - (double)s.lo[k];
    return e[0] * e[1] + e[1] * e[2] + e[2] * e[0];
  };
  // Which binary nodes become 4-wide nodes.  Default: the collapse that minimises the summed
  // surface area of the 4-wide nodes (the SAH traversal cost; the leaves and their cost are
  // fixed): f(n, k) = least area of 4-wide roots covering n's subtree with at most k slots,
  // f(n, 1) = A(n) + min_j f(L, j) + f(R, 4 - j), f(n, k) = min(f(n, 1), min_j f(L, j) + f(R, k - j)).
  // RT_COLLAPSE=greedy: open the largest-area internal slot until there are four.
  const char* ce = knob("RT_COLLAPSE");
  const bool greedy = ce && strcmp(ce, "greedy") == 0;
  const size_t nb = T->size();
  std::vector<double> f(nb * 5, 0.0);
  std::vector<signed char> split(nb * 5, 0);  // 0: keep the node as one slot, j > 0: j slots to the left
  auto fr = [&](int r, int k) -> double { return is_leaf(r) ? 0.0 : f[(size_t)r * 5 + k]; };
  if (!greedy && !is_leaf(croot)) {
    std::function<void(int)> dp = [&](int b) {
      Slot L, R;
      kids(b, L, R);
      if (!is_leaf(L.ref)) dp(L.ref);
      if (!is_leaf(R.ref)) dp(R.ref);
      Slot U = L;
      for (int k = 0; k < 3; k++) { U.lo[k] = std::min(L.lo[k], R.lo[k]); U.hi[k] = std::max(L.hi[k], R.hi[k]); }
      double open = 1e300;
      int jo = 1;
      for (int j = 1; j <= 3; j++) {
        const double c = fr(L.ref, j) + fr(R.ref, 4 - j);
        if (c < open) { open = c; jo = j; }
      }
      f[(size_t)b * 5 + 1] = area(U) + open;
      split[(size_t)b * 5 + 1] = (signed char)jo;  // the split of the node's own 4-wide record
      for (int k = 2; k <= 4; k++) {
        double best = f[(size_t)b * 5 + 1];
        int bj = 0;
        for (int j = 1; j < k; j++) {
          const double c = fr(L.ref, j) + fr(R.ref, k - j);
          if (c < best) { best = c; bj = j; }
        }
        f[(size_t)b * 5 + k] = best;
        split[(size_t)b * 5 + k] = (signed char)bj;
      }
    };
    dp(croot);
  }
  // DP reconstruction: the slots that binary subtree s contributes when given k of them
  std::function<void(const Slot&, int, std::vector<Slot>&)> collect = [&](const Slot& s, int k, std::vector<Slot>& out) {
    if (is_leaf(s.ref) || k == 1 || split[(size_t)s.ref * 5 + k] == 0) { out.push_back(s); return; }
    const int j = split[(size_t)s.ref * 5 + k];
    Slot L, R;
    kids(s.ref, L, R);
    collect(L, j, out);
    collect(R, k - j, out);
  };
  qdepth = 1;
  std::function<int(int, int)> build = [&](int b, int depth) -> int {
    qdepth = std::max(qdepth, depth);
    const int idx = (int)qn.size();
    qn.push_back(rtd::QNode{});
    std::vector<Slot> sl;
    if (greedy) {
      sl.resize(2);
      kids(b, sl[0], sl[1]);
      while (sl.size() < 4) {
        int pick = -1;
        double pa = -1.0;
        for (size_t i = 0; i < sl.size(); i++)
          if (!is_leaf(sl[i].ref) && area(sl[i]) > pa) { pa = area(sl[i]); pick = (int)i; }
        if (pick < 0) break;
        Slot x, y;
        kids(sl[pick].ref, x, y);
        sl[pick] = x;
        sl.insert(sl.begin() + pick + 1, y);
      }
    } else {
      Slot L, R;
      kids(b, L, R);
      const int j = split[(size_t)b * 5 + 1];
      collect(L, j, sl);
      collect(R, 4 - j, sl);
    }
    int refs[4] = {rtd::Q_EMPTY, rtd::Q_EMPTY, rtd::Q_EMPTY, rtd::Q_EMPTY};
    for (size_t i = 0; i < sl.size(); i++) refs[i] = is_leaf(sl[i].ref) ? sl[i].ref : build(sl[i].ref, depth + 1);
    // an empty slot is the inverted box lo = +inf, hi = -inf: for a finite 1/d the sign-selected
    // planes give entry t0 = +inf and exit t1 = -inf, so the slab test never hits it (the literal
    // slab of a ray with a zero direction component tests the slot's ref instead: its per-axis
    // min / max would turn the inverted box into an infinite one)
    const float pinf = INFINITY;
    float lo[3][4], hi[3][4];
    for (int k = 0; k < 3; k++)
      for (int i = 0; i < 4; i++) {
        lo[k][i] = i < (int)sl.size() ? sl[i].lo[k] : pinf;
        hi[k][i] = i < (int)sl.size() ? sl[i].hi[k] : -pinf;
      }
    rtd::QNode& q = qn[idx];
    q.lox = make_float4(lo[0][0], lo[0][1], lo[0][2], lo[0][3]);
    q.loy = make_float4(lo[1][0], lo[1][1], lo[1][2], lo[1][3]);
    q.loz = make_float4(lo[2][0], lo[2][1], lo[2][2], lo[2][3]);
    q.hix = make_float4(hi[0][0], hi[0][1], hi[0][2], hi[0][3]);
    q.hiy = make_float4(hi[1][0], hi[1][1], hi[1][2], hi[1][3]);
    q.hiz = make_float4(hi[2][0], hi[2][1], hi[2][2], hi[2][3]);
    q.ref = make_int4(refs[0], refs[1], refs[2], refs[3]);
    return idx;
  };
  qroot = is_leaf(croot) ? croot : build(croot, 1);
  const char* qb = knob("RT_QBFS");
  if (!is_leaf(qroot) && !(qb && atoi(qb) == 0)) {
    // breadth-first numbering (RT_QBFS=0: depth-first): the top levels of the tree are the
    // first nodes (RT_DEBUG_PASSES reports node visits by this index)
    std::vector<int> order{qroot}, newid(qn.size(), -1);
    newid[qroot] = 0;
    for (size_t h = 0; h < order.size(); h++) {
      const int4 r = qn[order[h]].ref;
      for (int x : {r.x, r.y, r.z, r.w})
        if (x != rtd::Q_EMPTY && !is_leaf(x)) {
          newid[x] = (int)order.size();
          order.push_back(x);
        }
    }
    std::vector<rtd::QNode> bq(order.size());
    auto remap = [&](int x) { return (x == rtd::Q_EMPTY || is_leaf(x)) ? x : newid[x]; };
    for (size_t i = 0; i < order.size(); i++) {
      bq[i] = qn[order[i]];
      bq[i].ref = make_int4(remap(bq[i].ref.x), remap(bq[i].ref.y), remap(bq[i].ref.z), remap(bq[i].ref.w));
    }
    qn.swap(bq);
    qroot = 0;
  }
  return true;
}

int upload(rt_ctx* c, void** dst, const void* src, size_t bytes) {
  if (*dst) { (void)hipFree(*dst); *dst = nullptr; }
  if (bytes == 0) return RT_OK;
  HIPCHK(c, hipMalloc(dst, bytes));
  HIPCHK(c, hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice));
  return RT_OK;
}

// Renders in flight read the scene, environment and pixel buffers: an entry point that replaces
// them first waits for them (the caller's stream joins every render call, pipelined ones too)
int drain(rt_ctx* c) {
  if (c->stream) HIPCHK(c, hipStreamSynchronize(c->stream));
  return RT_OK;
}

int occupancy(rt_ctx* c) {
  int lds = c->stack_entries * 256 * 8;
  int bpc = 0;
  HIPCHK(c, hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, rtd::rt_path_kernel<false>, 256, lds));
  c->blocks_per_cu = std::max(1, bpc);
  c->block_lds = lds;
  // wavefront traversal: short LDS stack + global overflow
  int kl = 8;  // 16 KiB per block: LDS leaves room for 8 waves/SIMD (12 entries: 6; C3 5853 -> 5959 at 10, 6155 at 8 with the dual schedule at 8 waves)
  if (const char* e = knob("RT_LDS_STACK")) kl = atoi(e);
  if (const char* e = knob("RT_SPLIT_KINDS")) c->split_kinds = atoi(e);
  if (const char* e = knob("RT_SPLIT_PASSES")) c->split_passes = atoi(e);
  kl = std::max(1, std::min(kl, std::max(c->stack_entries, c->qstack_entries)));
  c->trace_lds_entries = kl;
  c->trace_lds = kl * 256 * 8;
  bpc = 0;
  // persistent grids: as many blocks as can be resident (the camera pass's instantiation and the
  // secondary passes' one may differ in registers)
  auto occ = [&](bool cam) {
    int b = 0;
    const hipError_t e =
        cam ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, rtd::wf_trace<false, true, true>, 256, c->trace_lds)
            : hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, rtd::wf_trace<false, true, false>, 256, c->trace_lds);
    return e == hipSuccess ? std::max(1, b) : 1;
  };
  c->trace_bpc0 = occ(true);  // pass 0 is the implicit camera pass
  c->trace_bpc = occ(false);
  bpc = c->trace_bpc;
  if (const char* e = knob("RT_TRACE_BPC")) c->trace_bpc0 = c->trace_bpc = std::max(1, atoi(e));
  if (const char* e = knob("RT_POOL_CHUNK")) c->pool_chunk = std::max(64, atoi(e) / 64 * 64);
  if (knob("RT_DEBUG"))
    fprintf(stderr, "[rt] trace: lds entries %d (%d B/block), occupancy API %d blocks/CU, using %d (pass 0: %d); "
            "megakernel %d\n", kl, c->trace_lds, bpc, c->trace_bpc, c->trace_bpc0, c->blocks_per_cu);
  {
    int b = 0;
    const hipError_t e = c->wide
        ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, rtd::wf_finish<true, true>, 256, c->trace_lds)
        : hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, rtd::wf_finish<true, false>, 256, c->trace_lds);
    // the finisher's lanes index the traversal overflow column: never more than the trace grid
    c->finish_bpc = std::max(1, std::min(e == hipSuccess ? b : 1, std::max(c->trace_bpc, c->trace_bpc0)));
    if (const char* fe = knob("RT_FINISH_BPC")) c->finish_bpc = std::max(1, std::min(c->finish_bpc, atoi(fe)));
    c->pipe_finish_bpc = 2;
    if (const char* fe = knob("RT_PIPE_FINISH_BPC")) c->pipe_finish_bpc = std::max(1, atoi(fe));
    c->pipe_finish_bpc = std::min(c->pipe_finish_bpc, c->finish_bpc);
    if (knob("RT_DEBUG"))
      fprintf(stderr, "[rt] wf_finish: occupancy API %d blocks/CU, using %d (pipelined calls %d)\n", b, c->finish_bpc,
              c->pipe_finish_bpc);
  }
  const size_t lanes = (size_t)c->n_cus * std::max(c->trace_bpc, c->trace_bpc0) * 256;
  const int entries = std::max(c->stack_entries, c->qstack_entries);
  const size_t need = (size_t)std::max(0, entries - kl) * lanes * sizeof(int2) * c->n_groups;
  if (need > c->stack_ovf_bytes) {
    dfree(c->d_stack_ovf);
    HIPCHK(c, hipMalloc(&c->d_stack_ovf, need));
    c->stack_ovf_bytes = need;
  }
  return RT_OK;
}

// The traversal stack's overflow indices, checked on the host before every launch that uses them
// (DESIGN.md §4, round 5): entry j in [KL, entries) of grid lane l of path-state set `set` lives at
// element set * ovf_group + (j - KL) * ovf_lanes + l, with ovf_lanes = trace grid blocks * 256 and
// l below that (the finisher's grid is never larger than the trace grid); a lane-quad move copies
// at most `entries` = the deepest stack of the scene's trees (3 * qdepth + 2 for the 4-wide one),
// passed to the kernels as KParams::stack_cap.
std::string ovf_layout_error(const rt_ctx* c, int set, unsigned int trace_grid_blocks) {
  const int entries = std::max(c->stack_entries, c->qstack_entries);
  const int kl = c->trace_lds_entries;
  const size_t rows = (size_t)std::max(0, entries - kl);
  const size_t lanes = (size_t)trace_grid_blocks * 256u;
  const size_t per_set = c->stack_ovf_bytes / sizeof(int2) / (size_t)std::max(1, c->n_groups);
  char buf[256];
  if (set < 0 || set >= c->n_groups) {
    snprintf(buf, sizeof buf, "overflow stack: path-state set %d of %d", set, c->n_groups);
    return buf;
  }
  if (rows > 0 && (!c->d_stack_ovf || rows * lanes > per_set)) {
    snprintf(buf, sizeof buf, "overflow stack: %zu rows x %zu lanes exceed %zu entries per set", rows, lanes, per_set);
    return buf;
  }
  if ((unsigned)(c->finish_bpc * c->n_cus) > trace_grid_blocks || c->pipe_finish_bpc > c->finish_bpc) {
    snprintf(buf, sizeof buf, "overflow stack: finisher grid %d x %d above the trace grid %u", c->finish_bpc,
             c->n_cus, trace_grid_blocks);
    return buf;
  }
  return std::string();
}

template <bool COUNT, bool WIDE>
void launch_trace_w(rt_ctx* c, dim3 grid, const rtd::WFParams& WP, hipStream_t st, bool small) {
  // pass 1 reads the 16-B rays pass 0 queued (WFState::org) in an instantiation of its own, so the
  // later passes' kernel carries none of it
  const bool p1 = !WP.cam_n && WP.pass == 1 && WP.p1_compact;
  if (small && !COUNT && WIDE) {  // static first shares of mid-size passes
    if (WP.cam_n)
      hipLaunchKernelGGL((rtd::wf_trace<false, true, true, true>), grid, dim3(256), c->trace_lds, st, WP);
    else if (p1)
      hipLaunchKernelGGL((rtd::wf_trace<false, true, false, true, true>), grid, dim3(256), c->trace_lds, st, WP);
    else
      hipLaunchKernelGGL((rtd::wf_trace<false, true, false, true>), grid, dim3(256), c->trace_lds, st, WP);
    return;
  }
  if (WP.split && !WP.cam_n && !COUNT && WIDE) {  // split queues: the shadow rays, then the continuations
    for (int k = 0; k < 2; k++) {
      const bool shadow = (k == 0) != (RT_SPLIT_CONT_FIRST != 0);
      if (p1 && shadow) hipLaunchKernelGGL((rtd::wf_trace<false, true, false, false, true, 2>), grid, dim3(256), c->trace_lds, st, WP);
      else if (p1) hipLaunchKernelGGL((rtd::wf_trace<false, true, false, false, true, 1>), grid, dim3(256), c->trace_lds, st, WP);
      else if (shadow) hipLaunchKernelGGL((rtd::wf_trace<false, true, false, false, false, 2>), grid, dim3(256), c->trace_lds, st, WP);
      else hipLaunchKernelGGL((rtd::wf_trace<false, true, false, false, false, 1>), grid, dim3(256), c->trace_lds, st, WP);
    }
    return;
  }
  if (WP.cam_n)
    hipLaunchKernelGGL((rtd::wf_trace<COUNT, WIDE, true>), grid, dim3(256), c->trace_lds, st, WP);
  else if (p1)
    hipLaunchKernelGGL((rtd::wf_trace<COUNT, WIDE, false, false, true>), grid, dim3(256), c->trace_lds, st, WP);
  else
    hipLaunchKernelGGL((rtd::wf_trace<COUNT, WIDE, false>), grid, dim3(256), c->trace_lds, st, WP);
}

template <bool COUNT>
void launch_trace_t(rt_ctx* c, dim3 grid, const rtd::WFParams& WP, hipStream_t st, bool small) {
  if (c->wide) launch_trace_w<COUNT, true>(c, grid, WP, st, small);
  else launch_trace_w<COUNT, false>(c, grid, WP, st, small);
}

// small: a frame group of at most finish_slots path slots (one frame per call)
void launch_trace(rt_ctx* c, bool count, dim3 grid, const rtd::WFParams& WP, hipStream_t st, bool small) {
  if (count) launch_trace_t<true>(c, grid, WP, st, small);
  else launch_trace_t<false>(c, grid, WP, st, small);
}

hipEvent_t take_event(rt_ctx* c) {
  if (!c->event_pool.empty()) {
    hipEvent_t e = c->event_pool.back();
    c->event_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

// Timing events of launches not yet folded into kernel_ms / trace_ms: a front end that never
// calls rt_synchronize (it waits on its own stream or events) would otherwise grow these lists
// without bound.  Past `cap` pending pairs, the oldest are waited for, folded and recycled.
// a finished render call's (start, end) events: its duration into acc_ms
int fold_pair(rt_ctx* c, const std::pair<hipEvent_t, hipEvent_t>& e, double& acc_ms) {
  float ms = 0.0f;
  HIPCHK(c, hipEventElapsedTime(&ms, e.first, e.second));
  acc_ms += ms;
  c->event_pool.push_back(e.first);
  c->event_pool.push_back(e.second);
  return RT_OK;
}
// a finished traversal launch: its duration into trace_ms and its interval into the union
// (rt_ctx::busy; pairs arrive in queue order)
int fold_trace(rt_ctx* c, const rt_ctx::TraceEv& e) {
  float ms = 0.0f, a = 0.0f;
  HIPCHK(c, hipEventElapsedTime(&ms, e.s, e.e));
  c->trace_ms += ms;
  if (c->busy_anchor) HIPCHK(c, hipEventElapsedTime(&a, c->busy_anchor, e.s));
  double lo = c->busy_anchor_t + (double)a, hi = lo + (double)std::max(ms, 0.0f);
  if (c->busy_anchor) c->event_pool.push_back(c->busy_anchor);
  c->busy_anchor = e.s;  // this launch's start is the next one's reference
  c->busy_anchor_t = lo;
  c->event_pool.push_back(e.e);
  auto& v = c->busy;
  // close what no pending launch can overlap any more (calls <= e.call - 2)
  size_t keep = 0;
  for (const auto& iv : v) {
    if (iv.call + 2 <= e.call) c->busy_closed_ms += iv.hi - iv.lo;
    else v[keep++] = iv;
  }
  v.resize(keep);
  // merge [lo, hi] into the sorted disjoint list
  uint64_t call = e.call;
  auto it = std::upper_bound(v.begin(), v.end(), lo, [](double x, const rt_ctx::BusyIv& iv) { return x < iv.lo; });
  if (it != v.begin() && std::prev(it)->hi >= lo) {
    --it;
    lo = it->lo;
    hi = std::max(hi, it->hi);
    call = std::max(call, it->call);
    it = v.erase(it);
  }
  while (it != v.end() && it->lo <= hi) {
    hi = std::max(hi, it->hi);
    call = std::max(call, it->call);
    it = v.erase(it);
  }
  v.insert(it, rt_ctx::BusyIv{lo, hi, call});
  return RT_OK;
}

// Past `cap` pending pairs, the oldest are waited for, folded and recycled.  Pairs of one call can
// sit on different streams (frame / pixel groups, pipelined sets), so each pair is waited for
// itself (in queue order: cheap once the first is done).
int fold_events(rt_ctx* c, std::vector<std::pair<hipEvent_t, hipEvent_t>>& ev, double& acc_ms, size_t cap) {
  if (ev.size() <= cap) return RT_OK;
  const size_t n = ev.size() - cap / 2;
  for (size_t i = 0; i < n; i++) {
    HIPCHK(c, hipEventSynchronize(ev[i].second));
    const int rc = fold_pair(c, ev[i], acc_ms);
    if (rc) return rc;
  }
  ev.erase(ev.begin(), ev.begin() + (ptrdiff_t)n);
  return RT_OK;
}
int fold_trace_events(rt_ctx* c, size_t cap) {
  auto& ev = c->trace_events;
  if (ev.size() <= cap) return RT_OK;
  const size_t n = ev.size() - cap / 2;
  for (size_t i = 0; i < n; i++) {
    HIPCHK(c, hipEventSynchronize(ev[i].e));
    const int rc = fold_trace(c, ev[i]);
    if (rc) return rc;
  }
  ev.erase(ev.begin(), ev.begin() + (ptrdiff_t)n);
  return RT_OK;
}
constexpr size_t kMaxPendingEvents = 4096;

// Frames in flight per launch = path-state budget / pixels of this rank.  The state grows on
// demand in rt_render_async, so interactive 1-frame use stays small.  More frames per launch
// amortise the per-pass latency floor of the few longest rays (C3 1080p: 16 frames 1.07, 64
// frames 0.94 ms/frame; 161 vs 80 frames +1.8%, all 512 of a bench step at once +2.2%).
void update_frames_cap(rt_ctx* c, size_t nv) {
  size_t max_slots = size_t(320) << 20;  // 184 B each: 62 GB of the 288 GB HBM3E
  if (const char* e = knob("RT_MAX_SLOTS")) max_slots = (size_t)strtoull(e, nullptr, 10);
  if (c->max_slots_req) max_slots = c->max_slots_req;
  c->frames_cap = (int)std::max<size_t>(1, std::min<size_t>(RT_MAX_FRAMES_PER_LAUNCH, max_slots / std::max<size_t>(1, nv)));
}

// Path-state buffers of the wavefront path: `paths` slots for each of the n_groups frame
// groups, carved from one allocation (184 B per slot + counters).  RT_ERR_NOMEM when HBM
// cannot hold them (the caller then runs fewer frames at a time).
static_assert(rt_ctx::MAX_GROUPS <= 4, "rtd::GroupCounters holds 4 groups' counters");
int alloc_wavefront(rt_ctx* c, size_t paths) {
  if (c->wf_mem && c->wf_paths >= paths) return RT_OK;
  if (c->wf_mem) {  // grow: earlier launches on the streams may still read the old state
    HIPCHK(c, hipDeviceSynchronize());
    (void)hipFree(c->wf_mem);
    c->wf_mem = nullptr;
  }
  const size_t P = std::max<size_t>(paths, 64);
  const size_t per = P * (5 * 16 + sizeof(*c->wfg[0].s5) + 2 * (16 + 8) + 2 * 4 + 16 + 2 * 8 + 2 * 4) + 32768;  // + carve padding
  const hipError_t me = hipMalloc(&c->wf_mem, per * c->n_groups);
  if (me == hipErrorOutOfMemory) {
    (void)hipGetLastError();
    c->wf_mem = nullptr;
    c->wf_paths = 0;
    return fail(c, RT_ERR_NOMEM, "path state does not fit in device memory");
  }
  HIPCHK(c, me);
  char* p = static_cast<char*>(c->wf_mem);
  auto carve = [&](size_t n) { char* q = p; p += (n + 255) & ~size_t(255); return q; };
  for (int g = 0; g < c->n_groups; g++) {
    rtd::WFState& w = c->wfg[g];
    w.s0 = (float4*)carve(P * 16); w.s1 = (float4*)carve(P * 16); w.s2 = (float4*)carve(P * 16);
    w.s3 = (float4*)carve(P * 16); w.s4 = (float4*)carve(P * 16); w.s5 = (decltype(w.s5))carve(P * sizeof(*w.s5));
    w.ra = (float4*)carve(P * 16); w.rb = (float2*)carve(P * 8);
    w.sa = (float4*)carve(P * 16); w.sb = (float2*)carve(P * 8);
    w.res = (int*)carve(P * 8);
    w.fin = (float4*)carve(P * 16);
    w.queue[0] = (int*)carve(P * 8); w.queue[1] = (int*)carve(P * 8);
    w.queue_s[0] = w.queue[0] + P; w.queue_s[1] = w.queue[1] + P;  // (split queues: one entry per path each)
    w.active[0] = (int*)carve(P * 4); w.active[1] = (int*)carve(P * 4);
    w.cnt = (unsigned int*)carve(rtd::kCntWords * 4);
  }
  c->wf_paths = P;
  return RT_OK;
}

}  // namespace

extern "C" {

int rt_create(int hip_device, rt_ctx** out) {
  if (!out) return RT_ERR_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return RT_ERR_NODEVICE;
  if (hip_device < 0 || hip_device >= n) return RT_ERR_NODEVICE;
  rt_ctx* c = new (std::nothrow) rt_ctx();
  if (!c) return RT_ERR_NOMEM;
  c->device = hip_device;
  if (hipSetDevice(hip_device) != hipSuccess) { delete c; return RT_ERR_HIP; }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, hip_device) != hipSuccess) { delete c; return RT_ERR_HIP; }
  c->n_cus = prop.multiProcessorCount;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) { delete c; return RT_ERR_HIP; }
  c->own_stream = true;
  if (const char* e = knob("RT_GROUPS")) c->n_groups = std::max(1, std::min(rt_ctx::MAX_GROUPS, atoi(e)));
  if (const char* e = knob("RT_FINISH_PASS")) c->finish_pass = std::max(0, atoi(e));
  if (const char* e = knob("RT_PIPE_FINISH_PASS")) c->pipe_finish_pass = std::max(0, atoi(e));
  if (const char* e = knob("RT_FINISH_SLOTS")) c->finish_slots = (uint64_t)strtoull(e, nullptr, 10);
  if (hipMalloc(&c->d_counter, 64) != hipSuccess || hipMalloc(&c->d_stats, rtd::kStatWords * sizeof(unsigned long long)) != hipSuccess ||
      hipMemset(c->d_stats, 0, rtd::kStatWords * sizeof(unsigned long long)) != hipSuccess) {
    rt_destroy(c);
    return RT_ERR_HIP;
  }
  *out = c;
  return RT_OK;
}

int rt_destroy(rt_ctx* c) {
  if (!c) return RT_ERR_ARG;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (auto& a : c->aux) if (a) (void)hipStreamSynchronize(a);
  for (auto& e : c->events) { (void)hipEventDestroy(e.first); (void)hipEventDestroy(e.second); }
  for (auto& e : c->set_free) if (e) (void)hipEventDestroy(e);
  if (c->batch_done) (void)hipEventDestroy(c->batch_done);
  if (c->busy_anchor) (void)hipEventDestroy(c->busy_anchor);
  dfree(c->d_nodes); dfree(c->d_qnodes); dfree(c->d_tri); dfree(c->d_trx); dfree(c->d_trin); dfree(c->d_hrec); dfree(c->d_mats);
  for (auto& t : c->light) {
    dfree(t.d);
    if (t.last_use) (void)hipEventDestroy(t.last_use);
    if (t.built) (void)hipEventDestroy(t.built);
  }
  dfree(c->d_hdr); dfree(c->d_cache); dfree(c->d_accum); dfree(c->d_counter); dfree(c->d_stats);
  for (auto& e : c->trace_events) { (void)hipEventDestroy(e.s); (void)hipEventDestroy(e.e); }
  for (auto e : c->event_pool) (void)hipEventDestroy(e);
  if (c->wf_mem) (void)hipFree(c->wf_mem);
  for (auto& a : c->aux) if (a) (void)hipStreamDestroy(a);
  for (auto& d : c->disp) {
    if (d.ev) (void)hipEventDestroy(d.ev);
    if (d.host) (void)hipHostFree(d.host);
  }
  for (auto& t : c->ft) {
    if (t.ev) (void)hipEventDestroy(t.ev);
    if (t.h) (void)hipHostFree(t.h);
    dfree(t.d);
  }
  dfree(c->d_pix);
  dfree(c->d_tile_ids);
  dfree(c->d_tile_src);
  dfree(c->d_tile_cost);
  dfree(c->d_cam);
  dfree(c->d_stack_ovf);
  dfree(c->d_disp);
  dfree(c->d_gather);
  for (auto& m : c->rccl_comms) (void)ncclCommDestroy(m);
  if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return RT_OK;
}

const char* rt_last_error(const rt_ctx* c) { return c ? c->err.c_str() : "null context"; }

int rt_device_info(const rt_ctx* c, int32_t* n_cus, int32_t* blocks_per_cu, int32_t* lds_bytes_per_block) {
  if (!c) return RT_ERR_ARG;
  if (n_cus) *n_cus = c->n_cus;
  if (blocks_per_cu) *blocks_per_cu = c->blocks_per_cu;
  if (lds_bytes_per_block) *lds_bytes_per_block = c->block_lds;
  return RT_OK;
}

int rt_set_scene(rt_ctx* c, const rt_scene_soa* s) {
  if (!c || !s) return RT_ERR_ARG;
  if (s->n_triangles < 0 || s->n_nodes < 0 || s->n_materials < 0) return fail(c, RT_ERR_ARG, "negative count");
  const int nt = s->n_triangles;
  if (nt > 0 && (!s->p1 || !s->p2 || !s->p3 || !s->n1 || !s->n2 || !s->n3 || !s->material_id || !s->materials))
    return fail(c, RT_ERR_ARG, "missing triangle arrays");
  if (nt >= (1 << 27)) return fail(c, RT_ERR_LIMIT, "more than 2^27 triangles");
  HIPCHK(c, hipSetDevice(c->device));
  if (int rc = drain(c)) return rc;
  for (int i = 0; i < nt; i++)
    if (s->material_id[i] < 0 || s->material_id[i] >= s->n_materials)
      return fail(c, RT_ERR_ARG, "material_id out of range");
  // ---- triangles
  std::vector<float4> tri(3 * (size_t)nt), trin(3 * (size_t)nt);
  for (int i = 0; i < nt; i++) {
    float ng[3];
    geometric_normal(s->p1 + 3 * i, s->p2 + 3 * i, s->p3 + 3 * i, ng);
    const float* ps[3] = {s->p1 + 3 * i, s->p2 + 3 * i, s->p3 + 3 * i};
    const float* ns[3] = {s->n1 + 3 * i, s->n2 + 3 * i, s->n3 + 3 * i};
    for (int k = 0; k < 3; k++) {
      tri[3 * i + k] = make_float4(ps[k][0], ps[k][1], ps[k][2], ng[k]);
      float w = 0.0f;
      if (k == 0) memcpy(&w, &s->material_id[i], 4);
      trin[3 * i + k] = make_float4(ns[k][0], ns[k][1], ns[k][2], w);
    }
  }
  // ---- materials
  std::vector<float> mt(32 * (size_t)std::max(1, s->n_materials), 0.0f);
  for (int m = 0; m < s->n_materials; m++) pack_material(s->materials[m], &mt[32 * m]);
  // ---- BVH: reference numbering -> children-in-parent nodes
  int root = 0, has = 0, depth = 1;
  std::vector<GNode> gn;
  if (nt > 0 && s->n_nodes > 1) {
    if (!s->node_left || !s->node_right || !s->node_n || !s->node_index || !s->node_aa || !s->node_bb)
      return fail(c, RT_ERR_ARG, "missing node arrays");
    const int nn = s->n_nodes;
    std::vector<int> internal_id(nn, -1);
    auto is_leaf = [&](int i) { return s->node_n[i] > 0; };
    auto leaf_ref = [&](int i, int& ref) -> int {
      int n = s->node_n[i], first = s->node_index[i];
      if (n > 16) return fail(c, RT_ERR_LIMIT, "leaf with more than 16 triangles");
      if (first < 0 || first + n > nt) return fail(c, RT_ERR_ARG, "leaf range outside the triangle list");
      ref = (int)(rtd::LEAF_BIT | ((uint32_t)first << 4) | (uint32_t)(n - 1));
      return RT_OK;
    };
    // DFS from the root (node 1) assigning internal ids, checking structure and depth
    std::vector<std::pair<int, int>> st;
    st.push_back({1, 1});
    std::vector<int> order;
    while (!st.empty()) {
      auto e = st.back();
      st.pop_back();
      int i = e.first;
      if (i <= 0 || i >= nn) return fail(c, RT_ERR_ARG, "child index out of range");
      depth = std::max(depth, e.second);
      if (depth > 64) return fail(c, RT_ERR_LIMIT, "BVH deeper than 64 levels");
      if (is_leaf(i)) continue;
      if (internal_id[i] >= 0) return fail(c, RT_ERR_ARG, "BVH is not a tree");
      if (s->node_left[i] <= 0 || s->node_right[i] <= 0) return fail(c, RT_ERR_ARG, "internal node without two children");
      internal_id[i] = (int)order.size();
      order.push_back(i);
      st.push_back({s->node_right[i], e.second + 1});
      st.push_back({s->node_left[i], e.second + 1});
    }
    gn.resize(std::max<size_t>(1, order.size()));
    for (size_t k = 0; k < order.size(); k++) {
      int i = order[k];
      int l = s->node_left[i], r = s->node_right[i];
      const float* la = s->node_aa + 3 * l; const float* lb = s->node_bb + 3 * l;
      const float* ra = s->node_aa + 3 * r; const float* rb = s->node_bb + 3 * r;
      GNode g;
      g.b0 = make_float4(la[0], la[1], la[2], lb[0]);
      g.b1 = make_float4(lb[1], lb[2], ra[0], ra[1]);
      g.b2 = make_float4(ra[2], rb[0], rb[1], rb[2]);
      int lr, rr;
      int rc;
      if (is_leaf(l)) { if ((rc = leaf_ref(l, lr))) return rc; } else lr = internal_id[l];
      if (is_leaf(r)) { if ((rc = leaf_ref(r, rr))) return rc; } else rr = internal_id[r];
      g.ref = make_int4(lr, rr, 0, 0);
      gn[k] = g;
    }
    if (is_leaf(1)) {
      int rc = leaf_ref(1, root);
      if (rc) return rc;
    } else {
      root = internal_id[1];
    }
    has = 1;
  }
  std::vector<rtd::QNode> qn;
  int qroot = root, qdepth = 1;
  bool wide = false;
  if (has) wide = build_wide(gn, root, trin, qn, qroot, qdepth);
  if (const char* e = knob("RT_BVH_WIDTH")) if (atoi(e) == 2) wide = false;
  if (gn.empty()) {
    GNode z;
    memset(&z, 0, sizeof(z));
    gn.push_back(z);
  }
  if (qn.empty()) qn.push_back(rtd::QNode{});
  int rc;
  if ((rc = upload(c, (void**)&c->d_qnodes, qn.data(), qn.size() * sizeof(rtd::QNode)))) return rc;
  c->n_qnodes = (int)qn.size();
  if ((rc = upload(c, (void**)&c->d_nodes, gn.data(), gn.size() * sizeof(GNode)))) return rc;
  if ((rc = upload(c, (void**)&c->d_tri, tri.data(), tri.size() * sizeof(float4)))) return rc;
  {  // traversal records: {p1, Ng.x} {R2, Ng.y} {R3, Ng.z} and the edge filter's margin
    std::vector<float4> trx(std::max<size_t>(3, tri.size()));
    const trif::Consts k = trif::build(reinterpret_cast<const float*>(tri.data()), nt, reinterpret_cast<float*>(trx.data()));
    if ((rc = upload(c, (void**)&c->d_trx, trx.data(), trx.size() * sizeof(float4)))) return rc;
    c->tri_k1 = k.k1; c->tri_k0 = k.k0; c->tri_flagged = k.flagged;
  }
  if ((rc = upload(c, (void**)&c->d_trin, trin.data(), trin.size() * sizeof(float4)))) return rc;
  {  // hit records: tri's three texels then trin's, one 128-B line per triangle
    std::vector<float4> hr(8 * std::max<size_t>(1, (size_t)nt), make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    for (size_t i = 0; i < (size_t)nt; i++)
      for (int k = 0; k < 3; k++) {
        hr[8 * i + k] = tri[3 * i + k];
        hr[8 * i + 3 + k] = trin[3 * i + k];
      }
    if ((rc = upload(c, (void**)&c->d_hrec, hr.data(), hr.size() * sizeof(float4)))) return rc;
  }
  if ((rc = upload(c, (void**)&c->d_mats, mt.data(), mt.size() * sizeof(float)))) return rc;
  c->n_tri = nt;
  c->n_mats = s->n_materials;
  c->root = root;
  c->has_scene = has;
  {
    const CullStats cs = cull_bound_stats(s);
    c->cull_R = cs.R; c->cull_K = cs.K; c->cull_off = cs.off;
  }
  c->stack_entries = std::max(2, depth + 1);
  c->wide = wide;
  c->qroot = qroot;
  c->qstack_entries = std::max(2, 3 * qdepth + 2);
  c->tri_mat.assign(s->material_id, s->material_id + nt);
  c->mat_table = mt;
  c->scene_set = true;
  return occupancy(c);
}

int rt_set_scene_encoded(rt_ctx* c, const float* tri_enc, int32_t n_triangles, const float* node_enc, int32_t n_nodes) {
  if (!c || n_triangles < 0 || n_nodes < 0 || (n_triangles && !tri_enc) || (n_nodes && !node_enc)) return RT_ERR_ARG;
  const size_t nt = (size_t)n_triangles;
  std::vector<float> p[6];
  for (auto& v : p) v.resize(3 * nt);
  std::vector<int32_t> mid(nt);
  std::vector<rt_material> mats;
  for (size_t i = 0; i < nt; i++) {
    const float* t = tri_enc + 42 * i;  // Triangle_encoded: 14 texels
    for (int k = 0; k < 6; k++) memcpy(&p[k][3 * i], t + 3 * k, 12);
    rt_material m;
    memcpy(&m, t + 18, sizeof(rt_material));
    int found = -1;
    for (size_t q = 0; q < mats.size(); q++)
      if (!memcmp(&mats[q], &m, sizeof(m))) { found = (int)q; break; }
    if (found < 0) { mats.push_back(m); found = (int)mats.size() - 1; }
    mid[i] = found;
  }
  std::vector<int32_t> L(n_nodes), R(n_nodes), N(n_nodes), I(n_nodes);
  std::vector<float> aa(3 * (size_t)n_nodes), bb(3 * (size_t)n_nodes);
  for (int i = 0; i < n_nodes; i++) {  // BVHNode_encoded: ints stored as floats (RT:224-230 casts)
    const float* nd = node_enc + 12 * (size_t)i;
    L[i] = (int)nd[0]; R[i] = (int)nd[1]; N[i] = (int)nd[3]; I[i] = (int)nd[4];
    memcpy(&aa[3 * i], nd + 6, 12);
    memcpy(&bb[3 * i], nd + 9, 12);
  }
  rt_scene_soa s;
  s.n_triangles = n_triangles;
  s.p1 = p[0].data(); s.p2 = p[1].data(); s.p3 = p[2].data();
  s.n1 = p[3].data(); s.n2 = p[4].data(); s.n3 = p[5].data();
  s.material_id = mid.data();
  s.materials = mats.data();
  s.n_materials = (int32_t)mats.size();
  s.n_nodes = n_nodes;
  s.node_left = L.data(); s.node_right = R.data(); s.node_n = N.data(); s.node_index = I.data();
  s.node_aa = aa.data(); s.node_bb = bb.data();
  return rt_set_scene(c, &s);
}

int rt_update_materials(rt_ctx* c, int32_t first, int32_t count, const rt_material* m) {
  if (!c || !m || first < 0 || count < 0) return RT_ERR_ARG;
  if (!c->scene_set) return fail(c, RT_ERR_STATE, "no scene");
  if ((int64_t)first + count > c->n_tri) return fail(c, RT_ERR_ARG, "range outside the triangle list");
  HIPCHK(c, hipSetDevice(c->device));
  if (int rc = drain(c)) return rc;
  float packed[32];
  pack_material(*m, packed);
  int id = -1;
  for (int k = 0; k < c->n_mats; k++)
    if (!memcmp(&c->mat_table[32 * k], packed, sizeof(packed))) { id = k; break; }
  if (id < 0) {
    id = c->n_mats;
    c->mat_table.resize(32 * (size_t)(id + 1));
    memcpy(&c->mat_table[32 * id], packed, sizeof(packed));
    c->n_mats++;
    int rc = upload(c, (void**)&c->d_mats, c->mat_table.data(), c->mat_table.size() * sizeof(float));
    if (rc) return rc;
  }
  for (int i = first; i < first + count; i++) c->tri_mat[i] = id;
  if (count > 0) {
    hipLaunchKernelGGL(rtd::rt_set_material_kernel, dim3((count + 255) / 256), dim3(256), 0, c->stream,
                       c->d_trin, c->d_hrec, first, count, id);
    HIPCHK(c, hipGetLastError());
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return RT_OK;
}

int rt_set_env(rt_ctx* c, const float* hdr, const float* cache, int32_t w, int32_t h, int32_t res) {
  if (!c || !hdr || !cache || w <= 0 || h <= 0) return RT_ERR_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  if (int rc = drain(c)) return rc;
  // {hdrMap.rgb, hdrCache.b} per texel (a direction's colour and pdf in one fetch) + hdrCache.rg
  std::vector<float4> a((size_t)w * h);
  std::vector<float2> b((size_t)w * h);
  for (size_t i = 0; i < a.size(); i++) {
    a[i] = make_float4(hdr[3 * i], hdr[3 * i + 1], hdr[3 * i + 2], cache[3 * i + 2]);
    b[i] = make_float2(cache[3 * i], cache[3 * i + 1]);
  }
  int rc;
  if ((rc = upload(c, (void**)&c->d_hdr, a.data(), a.size() * sizeof(float4)))) return rc;
  if ((rc = upload(c, (void**)&c->d_cache, b.data(), b.size() * sizeof(float2)))) return rc;
  for (auto& t : c->light) {  // (drained above: no call reads them)
    dfree(t.d);
    HIPCHK(c, hipMalloc(&t.d, a.size() * 2 * sizeof(float4)));
    t.valid = false;
  }
  c->hdr_w = w; c->hdr_h = h; c->hdr_res = res;
  c->env_set = true;
  return RT_OK;
}

// (Re)build everything that depends on the tiling: the tile tables, the accumulation buffer
// (zeroed), this rank's pixel list (its tiles in local order, 8x8 blocks inside a tile: ray
// coherence) and the wavefront state sized for it.
static int apply_tiling(rt_ctx* c, int width, int height, const rt_tiling& tl, std::vector<int32_t> owner) {
  HIPCHK(c, hipSetDevice(c->device));
  if (int rc = drain(c)) return rc;  // renders in flight read the buffers replaced below
  // the old pixel lists / accumulation no longer describe the frame from here on: a failure
  // below leaves the context un-sized (rt_render_async then refuses) rather than half-resized
  c->frame_set = false;
  c->W = width; c->H = height;
  c->tile_w = tl.tile_w; c->tile_h = tl.tile_h; c->rank = tl.rank; c->world = tl.world;
  c->tiles_x = (width + tl.tile_w - 1) / tl.tile_w;
  c->tiles_y = (height + tl.tile_h - 1) / tl.tile_h;
  const int total = c->tiles_x * c->tiles_y;
  std::vector<int> count(tl.world, 0);
  std::vector<int2> src(total);
  c->my_tiles.clear();
  for (int t = 0; t < total; t++) {
    src[t] = make_int2(owner[t], count[owner[t]]++);
    if (owner[t] == tl.rank) c->my_tiles.push_back(t);
  }
  c->owner = std::move(owner);
  c->local_tiles = (int)c->my_tiles.size();
  c->max_local_tiles = *std::max_element(count.begin(), count.end());
  dfree(c->d_accum);
  size_t bytes = (size_t)std::max(1, c->max_local_tiles) * tl.tile_w * tl.tile_h * sizeof(float4);
  HIPCHK(c, hipMalloc(&c->d_accum, bytes));
  HIPCHK(c, hipMemset(c->d_accum, 0, bytes));
  dfree(c->d_tile_ids);
  dfree(c->d_tile_src);
  dfree(c->d_tile_cost);
  HIPCHK(c, hipMalloc(&c->d_tile_ids, std::max<size_t>(1, c->my_tiles.size()) * sizeof(int)));
  HIPCHK(c, hipMalloc(&c->d_tile_src, std::max<size_t>(1, src.size()) * sizeof(int2)));
  if (!c->my_tiles.empty())
    HIPCHK(c, hipMemcpy(c->d_tile_ids, c->my_tiles.data(), c->my_tiles.size() * sizeof(int), hipMemcpyHostToDevice));
  if (!src.empty()) HIPCHK(c, hipMemcpy(c->d_tile_src, src.data(), src.size() * sizeof(int2), hipMemcpyHostToDevice));
  std::vector<unsigned int> xy, acc;
  const int tpx = tl.tile_w * tl.tile_h;
  for (int lt = 0; lt < c->local_tiles; lt++) {
    const int gt = c->my_tiles[lt];
    const int tx = gt % c->tiles_x, ty = gt / c->tiles_x;
    for (int r = 0; r < tpx; r++) {
      const int blk = r >> 6, in = r & 63, bxs = tl.tile_w >> 3;
      const int lx = (blk % bxs) * 8 + (in & 7), ly = (blk / bxs) * 8 + (in >> 3);
      const int px = tx * tl.tile_w + lx, py = ty * tl.tile_h + ly;
      if (px >= width || py >= height) continue;
      xy.push_back((unsigned)px | ((unsigned)py << 16));
      acc.push_back((unsigned)(lt * tpx + ly * tl.tile_w + lx));
    }
  }
  c->n_valid = (int)xy.size();
  c->order_head = 0;
  dfree(c->d_pix);
  dfree(c->d_cam);
  const size_t nv = std::max<size_t>(1, xy.size());
  HIPCHK(c, hipMalloc(&c->d_pix, 2 * nv * sizeof(unsigned int)));
  HIPCHK(c, hipMalloc(&c->d_cam, 2 * nv * sizeof(float4)));
  c->cam_sets = 1;
  if (!xy.empty()) {
    HIPCHK(c, hipMemcpy(c->d_pix, xy.data(), xy.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->d_pix + nv, acc.data(), acc.size() * 4, hipMemcpyHostToDevice));
  }
  update_frames_cap(c, nv);
  int rc = alloc_wavefront(c, nv);
  if (rc) return rc;
  c->wf.pix_xy = c->d_pix;
  c->wf.pix_acc = c->d_pix + nv;
  c->wf.cam = c->d_cam;
  c->frame_set = true;
  c->loop_num = 0;
  return RT_OK;
}

int rt_resize(rt_ctx* c, int32_t width, int32_t height, const rt_tiling* t) {
  if (!c || width <= 0 || height <= 0) return RT_ERR_ARG;
  rt_tiling tl = t ? *t : rt_tiling{32, 32, 0, 1};
  if (tl.tile_w <= 0 || tl.tile_h <= 0 || (tl.tile_w % 8) || (tl.tile_h % 8) || tl.world <= 0 || tl.rank < 0 ||
      tl.rank >= tl.world)
    return fail(c, RT_ERR_ARG, "bad tiling (tile sizes must be positive multiples of 8, 0 <= rank < world)");
  if (width > 65535 || height > 65535) return fail(c, RT_ERR_LIMIT, "frame larger than 65535");
  const int total = ((width + tl.tile_w - 1) / tl.tile_w) * ((height + tl.tile_h - 1) / tl.tile_h);
  std::vector<int32_t> owner(total);
  for (int g = 0; g < total; g++) owner[g] = g % tl.world;  // interleaved default
  return apply_tiling(c, width, height, tl, std::move(owner));
}

int rt_set_tile_owners(rt_ctx* c, const int32_t* owner, int32_t n_tiles) {
  if (!c || !owner || n_tiles <= 0) return RT_ERR_ARG;
  if (!c->frame_set) return fail(c, RT_ERR_STATE, "rt_resize first");
  if (n_tiles != c->tiles_x * c->tiles_y) return fail(c, RT_ERR_ARG, "n_tiles differs from the frame's tile count");
  for (int g = 0; g < n_tiles; g++)
    if (owner[g] < 0 || owner[g] >= c->world) return fail(c, RT_ERR_ARG, "tile owner outside [0, world)");
  const rt_tiling tl{c->tile_w, c->tile_h, c->rank, c->world};
  return apply_tiling(c, c->W, c->H, tl, std::vector<int32_t>(owner, owner + n_tiles));
}

int rt_get_tile_owners(const rt_ctx* c, int32_t* owner, int32_t n_tiles) {
  if (!c || !owner) return RT_ERR_ARG;
  if (!c->frame_set) return RT_ERR_STATE;
  if (n_tiles != (int32_t)c->owner.size()) return RT_ERR_ARG;
  memcpy(owner, c->owner.data(), c->owner.size() * sizeof(int32_t));
  return RT_OK;
}

int rt_reset(rt_ctx* c) {
  if (!c) return RT_ERR_ARG;
  c->loop_num = 0;
  return RT_OK;
}
int rt_set_loop_num(rt_ctx* c, int32_t n) {
  if (!c || n < 0) return RT_ERR_ARG;
  c->loop_num = n;
  return RT_OK;
}
int rt_set_max_paths(rt_ctx* c, uint64_t slots) {
  if (!c) return RT_ERR_ARG;
  c->max_slots_req = (size_t)slots;
  if (c->frame_set) update_frames_cap(c, (size_t)c->n_valid);
  return RT_OK;
}

int rt_get_loop_num(const rt_ctx* c, int32_t* n) {
  if (!c || !n) return RT_ERR_ARG;
  *n = c->loop_num;
  return RT_OK;
}
int rt_set_finish(rt_ctx* c, int32_t pass, uint64_t max_slots) {
  if (!c || pass < 0) return RT_ERR_ARG;
  c->finish_pass = pass;
  c->finish_slots = max_slots;
  return RT_OK;
}

int rt_set_pipeline(rt_ctx* c, int32_t depth) {
  if (!c || depth < 1) return RT_ERR_ARG;
  int rc = rt_synchronize(c);  // calls in flight keep the sets they were given
  if (rc) return rc;
  c->pipe_depth = std::min<int>(depth, 2);  // streams aux[1], aux[2]
  c->pipe_next = 0;
  return RT_OK;
}

int rt_clear_accum(rt_ctx* c) {
  if (!c) return RT_ERR_ARG;
  if (!c->frame_set) return fail(c, RT_ERR_STATE, "rt_resize first");
  HIPCHK(c, hipSetDevice(c->device));
  size_t bytes = (size_t)std::max(1, c->max_local_tiles) * c->tile_w * c->tile_h * sizeof(float4);
  HIPCHK(c, hipMemsetAsync(c->d_accum, 0, bytes, c->stream));
  return RT_OK;
}

int rt_render_async(rt_ctx* c, const rt_frame_params* fp, const float* rand_origin, int32_t n_frames) {
  if (!c || !fp || n_frames < 0 || (n_frames && !rand_origin)) return RT_ERR_ARG;
  if (!c->scene_set || !c->env_set || !c->frame_set) return fail(c, RT_ERR_STATE, "set_scene, set_env and resize first");
  if ((fp->flags & RT_FLAG_MEGAKERNEL) && !fp->enable_bsdf)
    return fail(c, RT_ERR_ARG, "BRDF mode (enable_bsdf = 0) runs on the wavefront path only");
  HIPCHK(c, hipSetDevice(c->device));
  // main.cpp:175: LoopNum++ while below maxIterations; frames at the cap copy history (R12).
  int n_trace_pre = 0;
  for (int k = 0, ln = c->loop_num; k < n_frames; k++) {
    if (fp->max_iterations == -1 || ln < fp->max_iterations) ln++;
    if (fp->max_iterations == -1 || ln < fp->max_iterations) n_trace_pre++;
  }
  // a pipelined call (rt_set_pipeline): see rt_ctx::pipe_depth.  One-frame calls, and calls of
  // one batch (at most frames_cap frames) whose whole path state fits in each set.
  static const bool pix_ok = !knob("RT_PIX_SPLIT") || atoi(knob("RT_PIX_SPLIT")) != 0;
  const int pipe_sets = std::min(c->pipe_depth, c->n_groups);
  const size_t nv = std::max<size_t>(1, (size_t)c->n_valid);
  const bool serial = (fp->flags & RT_FLAG_SERIAL) != 0 && !(fp->flags & RT_FLAG_MEGAKERNEL);
  bool pipe = pipe_sets >= 2 && !(fp->flags & RT_FLAG_MEGAKERNEL) && !serial && n_trace_pre > 0 &&
              c->n_valid >= 64 * c->n_groups && !c->tile_cost_on &&
              (n_trace_pre < c->n_groups ||
               (n_trace_pre <= c->frames_cap && (size_t)n_trace_pre * nv < c->pipe_nomem_slots));
  if (pipe && n_trace_pre < c->n_groups && pix_ok) {
    // a one-frame call with no call in flight has nothing to overlap: the pixel-split groups
    // (below) have the lower latency (C4 1080p 5.6 vs 6.8 ms synchronised)
    bool idle = !(c->batch_done && hipEventQuery(c->batch_done) != hipSuccess);
    for (int q = 0; q < pipe_sets && idle; q++)
      if (c->set_free[q] && hipEventQuery(c->set_free[q]) != hipSuccess) idle = false;
    (void)hipGetLastError();  // (hipErrorNotReady is a status, not an error)
    if (idle) pipe = false;
  }
  if (!(fp->flags & RT_FLAG_MEGAKERNEL) && n_frames > 0) {
    int rc = RT_ERR_NOMEM;
    if (pipe && n_trace_pre >= c->n_groups) {  // a pipelined batch: the whole call in one set
      rc = alloc_wavefront(c, (size_t)n_trace_pre * nv);
      if (rc == RT_ERR_NOMEM) {  // not both sets: this size runs as frame groups from now on
        c->pipe_nomem_slots = std::min(c->pipe_nomem_slots, (size_t)n_trace_pre * nv);
        pipe = false;
      } else if (rc) {
        return rc;
      }
    }
    while (rc == RT_ERR_NOMEM) {  // a budget larger than free HBM runs fewer frames at a time
      const int per_group = (std::min(c->frames_cap, (int)n_frames) + c->n_groups - 1) / c->n_groups;
      rc = alloc_wavefront(c, (size_t)per_group * nv);
      if (rc != RT_ERR_NOMEM || per_group <= 1) break;
      c->frames_cap = std::max(1, std::min(c->frames_cap, (int)n_frames) / 2);
    }
    if (rc) return rc;
    for (int g = 1; g < c->n_groups; g++)
      if (!c->aux[g]) HIPCHK(c, hipStreamCreateWithFlags(&c->aux[g], hipStreamNonBlocking));
  }
  const int pset = pipe ? c->pipe_next : 0;
  // the stream that runs this call: pipelined sets on aux[1], aux[2] (aux[1] is also the second
  // frame group's stream: a pipelined call waits for unpipelined ones anyway, and a fourth stream
  // measured as losing the overlap, GPU_MAX_HW_QUEUES being 4)
  hipStream_t ps = pipe ? c->aux[1 + pset] : c->stream;
  hipEvent_t e_entry = nullptr;  // pipelined: the caller's stream at entry (the blend waits for it)
  if (pipe) {
    c->pipe_next = (c->pipe_next + 1) % pipe_sets;
    if (!ps) {
      HIPCHK(c, hipStreamCreateWithFlags(&c->aux[1 + pset], hipStreamNonBlocking));
      ps = c->aux[1 + pset];
    }
    if (c->cam_sets < pipe_sets) {  // one camera table per set (a call may move the camera)
      HIPCHK(c, hipStreamSynchronize(c->stream));
      dfree(c->d_cam);
      HIPCHK(c, hipMalloc(&c->d_cam, 2 * (size_t)std::max(1, c->n_valid) * pipe_sets * sizeof(float4)));
      c->cam_sets = pipe_sets;
      c->wf.cam = c->d_cam;
    }
    e_entry = take_event(c);
    if (!e_entry) return fail(c, RT_ERR_HIP, "hipEventCreate failed");
    HIPCHK(c, hipEventRecord(e_entry, c->stream));
    // the set's previous call and the last batched call have finished with its state
    if (c->set_free[pset]) HIPCHK(c, hipStreamWaitEvent(ps, c->set_free[pset], 0));
    if (c->batch_done) HIPCHK(c, hipStreamWaitEvent(ps, c->batch_done, 0));
  }
  // The traced frames' (loopNum, randOrigin) go to a device table in one upload.
  rt_ctx::FrameTable& T = c->ft[pipe ? 1 + pset : 0];
  if (n_frames > 0 && (size_t)n_frames > T.cap) {
    if (T.ev) HIPCHK(c, hipEventSynchronize(T.ev));
    if (T.h) (void)hipHostFree(T.h);
    T.h = nullptr;
    if (T.d) HIPCHK(c, hipStreamSynchronize(c->stream));  // calls in flight read the old table
    dfree(T.d);
    const size_t cap = std::max<size_t>(pipe ? 16 : 1024, (size_t)n_frames);
    HIPCHK(c, hipHostMalloc((void**)&T.h, 2 * cap * sizeof(int)));
    // device table: [cap] loop_num, [cap] rand_origin, then [cap][4] float2 Sobol pairs and [cap]
    // float2 blend weights (wf_sobol)
    HIPCHK(c, hipMalloc((void**)&T.d, 12 * cap * sizeof(int)));
    T.cap = cap;
  }
  if (!T.ev) HIPCHK(c, hipEventCreateWithFlags(&T.ev, hipEventDisableTiming));
  HIPCHK(c, hipEventSynchronize(T.ev));  // the previous upload from this table has read T.h
  int n_traced = 0;
  for (int k = 0; k < n_frames; k++) {
    if (fp->max_iterations == -1 || c->loop_num < fp->max_iterations) c->loop_num++;
    if (!(fp->max_iterations == -1 || c->loop_num < fp->max_iterations)) continue;
    T.h[n_traced] = c->loop_num;
    memcpy(&T.h[T.cap + n_traced], &rand_origin[k], 4);
    n_traced++;
  }
  // small calls hand the pairs to wf_sobol as kernel arguments, which writes the table
  rtd::InlineFrames IF;
  memset(&IF, 0, sizeof(IF));
  if (n_traced > 0 && n_traced <= RT_INLINE_FRAMES && !(fp->flags & RT_FLAG_MEGAKERNEL)) {
    IF.n_inline = n_traced;
    for (int k = 0; k < n_traced; k++) {
      IF.loop[k] = T.h[k];
      memcpy(&IF.ro[k], &T.h[T.cap + k], 4);
    }
  } else if (n_traced > 0) {
    HIPCHK(c, hipMemcpyAsync(T.d, T.h, (size_t)n_traced * sizeof(int), hipMemcpyHostToDevice, ps));
    HIPCHK(c, hipMemcpyAsync(T.d + T.cap, T.h + T.cap, (size_t)n_traced * sizeof(int), hipMemcpyHostToDevice, ps));
  }
  HIPCHK(c, hipEventRecord(T.ev, ps));
  const int* d_loop = T.d;
  const float* d_ro = reinterpret_cast<const float*>(T.d + T.cap);
  float2* d_sobol = reinterpret_cast<float2*>(T.d + 2 * T.cap);
  float2* d_blendw = reinterpret_cast<float2*>(T.d + 10 * T.cap);
  if (n_traced > 0 && !(fp->flags & RT_FLAG_MEGAKERNEL)) {
    hipLaunchKernelGGL(rtd::wf_sobol, dim3((4 * n_traced + 255) / 256), dim3(256), 0, ps, T.d,
                       reinterpret_cast<float*>(T.d + T.cap), d_sobol, d_blendw, n_traced, IF);
    HIPCHK(c, hipGetLastError());
  }
  // NEE light table for this call's envAngle (SampleHdrLight): the table built for this angle, or
  // the other one rebuilt on this call's stream once the last call that read it has finished (a
  // device-side wait: an interactive envAngle drag keeps its frames in flight)
  rt_ctx::LightTable* LT = &c->light[c->light_cur];
  if (n_traced > 0 && !(fp->flags & RT_FLAG_MEGAKERNEL)) {
    auto same = [&](const rt_ctx::LightTable& t) {
      return t.valid && __builtin_memcmp(&t.angle, &fp->env_angle, sizeof(float)) == 0;
    };
    if (!same(*LT)) {
      const int other = c->light_cur ^ 1;
      LT = &c->light[other];
      c->light_cur = other;
      if (!same(*LT)) {
        if (LT->last_use) HIPCHK(c, hipStreamWaitEvent(ps, LT->last_use, 0));
        const rtd::Env E{c->d_hdr, c->d_cache, LT->d, c->hdr_w, c->hdr_h, c->hdr_res, fp->env_angle, fp->env_intensity};
        const unsigned int n = (unsigned int)(c->hdr_w * c->hdr_h);
        hipLaunchKernelGGL(rtd::rt_light_table_kernel, dim3(std::max(1u, std::min(4096u, (n + 255) / 256))), dim3(256),
                           0, ps, E, LT->d);
        HIPCHK(c, hipGetLastError());
        if (!LT->built) HIPCHK(c, hipEventCreateWithFlags(&LT->built, hipEventDisableTiming));
        HIPCHK(c, hipEventRecord(LT->built, ps));
        LT->angle = fp->env_angle;
        LT->valid = true;
      }
    }
    // every call that reads the table waits for its build, which may still run on another call's
    // stream (a pipelined call on aux[1] rebuilt it; this one runs on aux[2] with the same angle)
    if (LT->built) HIPCHK(c, hipStreamWaitEvent(ps, LT->built, 0));
  }
  int done = 0;
  while (done < n_traced) {
    KParams P;
    memset(&P, 0, sizeof(P));
    // RT_FLAG_SERIAL: one frame group per batch, as many frames as one group's path state holds
    const int cap = (fp->flags & RT_FLAG_MEGAKERNEL) ? RT_MAX_FRAMES_PER_LAUNCH
                    : serial ? (int)std::max<size_t>(1, std::min<size_t>((size_t)c->frames_cap, c->wf_paths / nv))
                             : c->frames_cap;
    const int nf = std::min(cap, n_traced - done);
    P.loop_num = d_loop + done;
    P.rand_origin = d_ro + done;
    P.sobol = d_sobol + 4 * (size_t)done;
    P.blend_w = d_blendw + done;
    done += nf;
    memcpy(P.pos, fp->position, 12); memcpy(P.lbc, fp->left_bottom_corner, 12);
    memcpy(P.right, fp->right, 12); memcpy(P.up, fp->up, 12);
    P.half_w = fp->half_w; P.half_h = fp->half_h;
    P.enable_mis = fp->enable_mis; P.enable_env = fp->enable_env_map; P.enable_bsdf = fp->enable_bsdf;
    P.env_intensity = fp->env_intensity; P.env_angle = fp->env_angle;
    P.max_bounce = fp->max_bounce; P.flags = fp->flags; P.n_frames = nf;
    P.W = c->W; P.H = c->H; P.tile_w = c->tile_w; P.tile_h = c->tile_h; P.tiles_x = c->tiles_x;
    P.rank = c->rank; P.world = c->world; P.tile_ids = c->d_tile_ids;
    P.tile_cost = c->tile_cost_on ? c->d_tile_cost : nullptr;
    P.cost_blocks = c->cost_blocks ? 1 : 0;
    P.n_work = (unsigned)c->local_tiles * (unsigned)(c->tile_w * c->tile_h);
    P.nodes = c->d_nodes; P.root = c->root; P.has_scene = c->has_scene; P.stack_entries = c->stack_entries;
    P.stack_cap = std::max(c->stack_entries, c->qstack_entries);
    P.qnodes = c->d_qnodes; P.qroot = c->qroot; P.n_qnodes = c->n_qnodes; P.n_tri = c->n_tri;
    {  // eps of the culling bound for this call's origins (camera position, scene points)
      double R = c->cull_R;
      for (int a = 0; a < 3; a++) R = std::max(R, std::fabs((double)fp->position[a]));
      // x (1 + 2^-9): the fp32 rounding of eps * max|1/d| and of the sum in cull_limit
      const double eps = 2.0 * (c->cull_K * 0x1p-24 * R * (1.0 + 0x1p-10) + c->cull_off) * (1.0 + 0x1p-9);
      // RT_CULL_EPS_SCALE (tests only): 0 restores the round-1 heuristic margin, whose hole
      // tests/test_gpu_cull.py demonstrates
      const char* es = knob("RT_CULL_EPS_SCALE");
      const double sc = es ? atof(es) : 1.0;
      P.cull_eps = (eps * sc < 1e30) ? (float)(eps * sc) : INFINITY;
    }
    P.tri = c->d_tri; P.trin = c->d_trin; P.hrec = c->d_hrec; P.mats = c->d_mats;
    {  // edge-filter margin, rounded up (x (1 + 2^-20)); RT_TRI_MARGIN_SCALE (tests only): 0 makes
       // the filter decide every point, the negative control of tests/test_gpu_tri_filter.py
      const char* ms = knob("RT_TRI_MARGIN_SCALE");
      const double sc = ms ? atof(ms) : 1.0;
      P.trx = c->d_trx;
      P.tri_k1 = (float)(c->tri_k1 * sc * (1.0 + 0x1p-20));
      P.tri_k0 = (float)(c->tri_k0 * sc * (1.0 + 0x1p-20));
    }
    P.hdr = c->d_hdr; P.cache = c->d_cache; P.light = LT->d;
    P.hdr_w = c->hdr_w; P.hdr_h = c->hdr_h; P.hdr_res = c->hdr_res;
    P.accum = c->d_accum; P.counter = c->d_counter; P.stats = c->d_stats;
    if (P.n_work == 0) continue;
    const bool count = (fp->flags & RT_FLAG_COUNT_VISITS) != 0;
    hipEvent_t e0 = take_event(c), e1 = take_event(c);
    if (!e0 || !e1) return fail(c, RT_ERR_HIP, "hipEventCreate failed");
    HIPCHK(c, hipEventRecord(e0, ps));
    if (fp->flags & RT_FLAG_MEGAKERNEL) {
      HIPCHK(c, hipMemsetAsync(c->d_counter, 0, 4, c->stream));
      unsigned int max_blocks = (P.n_work + 255) / 256;
      unsigned int grid = std::min<unsigned int>((unsigned)(c->n_cus * c->blocks_per_cu), max_blocks);
      if (count)
        hipLaunchKernelGGL(rtd::rt_path_kernel<true>, dim3(grid), dim3(256), c->block_lds, c->stream, P);
      else
        hipLaunchKernelGGL(rtd::rt_path_kernel<false>, dim3(grid), dim3(256), c->block_lds, c->stream, P);
      HIPCHK(c, hipGetLastError());
      c->trace_launches++;
    } else {
      // split the batch into frame groups (frames [f0, f1) each), one stream per group; a batch
      // of fewer frames than groups (one frame per call: the reference's own usage) is split by
      // pixels instead (work items [w0, w1) each, all frames), so the groups' latency-bound late
      // passes still overlap each other
      const bool pix_split = !pipe && !serial && pix_ok && nf < c->n_groups && c->n_valid >= 64 * c->n_groups && !c->tile_cost_on;
      const int G = (pipe || serial) ? 1 : pix_split ? c->n_groups : std::min(c->n_groups, nf);
      const unsigned int trace_grid = (unsigned)(c->n_cus * std::max(c->trace_bpc, c->trace_bpc0));
      const unsigned int trace_grid0 = (unsigned)(c->n_cus * c->trace_bpc0);
      const unsigned int trace_grid1 = (unsigned)(c->n_cus * c->trace_bpc);
#ifdef RT_DEV  // RT_DEBUG_PASSES: per-pass report of the COUNT build (syncs after every pass)
      static const bool debug_passes = knob("RT_DEBUG_PASSES") != nullptr;
      static unsigned long long* d_wave_log = nullptr;  // never freed
      std::vector<unsigned long long> wave_log;
      if (debug_passes) {
        if (!d_wave_log) HIPCHK(c, hipMalloc(&d_wave_log, (size_t)trace_grid * 4 * 8 * sizeof(unsigned long long)));
        wave_log.resize((size_t)trace_grid * 4 * 8);  // (the trace's records use the first half)
      }
#else
      constexpr bool debug_passes = false;
      unsigned long long* d_wave_log = nullptr;
#endif
      const size_t ovf_group = c->stack_ovf_bytes / sizeof(int2) / (size_t)c->n_groups;
      rtd::WFParams WG[rt_ctx::MAX_GROUPS];
      hipStream_t sg[rt_ctx::MAX_GROUPS];
      unsigned int slots_g[rt_ctx::MAX_GROUPS];
      int split_g[rt_ctx::MAX_GROUPS] = {};
      // pixel ranges of the groups: even, or after rt_order_work the costly head as group 0 and
      // the rest split evenly (dev: RT_GROUP_SPLIT = group 0's share)
      size_t b0 = std::min(c->order_head, (size_t)c->n_valid);
#ifdef RT_DEV
      if (const char* e = knob("RT_GROUP_SPLIT")) b0 = std::min((size_t)c->n_valid, ((size_t)((double)c->n_valid * atof(e)) + 63) / 64 * 64);
#endif
      auto wbound = [&](int g) -> unsigned int {
        if (g <= 0) return 0u;
        if (g >= G) return (unsigned)c->n_valid;
        if (b0 > 0 && G > 1) return (unsigned)(b0 + ((size_t)c->n_valid - b0) * (g - 1) / (G - 1));
        return (unsigned)((size_t)c->n_valid * g / G);
      };
      for (int g = 0; g < G; g++) {
        const int f0 = pix_split ? 0 : g * nf / G, f1 = pix_split ? nf : (g + 1) * nf / G;
        const unsigned int w0 = pix_split ? wbound(g) : 0u;
        const unsigned int w1 = pix_split ? wbound(g + 1) : (unsigned)c->n_valid;
        rtd::WFParams& WP = WG[g];
        WP.K = P;
        WP.K.loop_num = P.loop_num + f0;
        WP.K.rand_origin = P.rand_origin + f0;
        WP.K.sobol = P.sobol + 4 * f0;
        WP.K.blend_w = P.blend_w + f0;
        WP.K.n_frames = f1 - f0;
        WP.K.n_work = w1 - w0;
        WP.K.lds_entries = c->trace_lds_entries;
        WP.K.pool_chunk = c->pool_chunk;
        const int set = pipe ? pset : g;  // path-state set, overflow column, stream
        float4* cam = c->wf.cam + (pipe ? (size_t)pset * (size_t)c->n_valid : 0);
        float4* org = c->wf.cam + (size_t)c->cam_sets * (size_t)std::max(1, c->n_valid) +
                      (pipe ? (size_t)pset * (size_t)c->n_valid : 0);
        WP.K.stack_ovf = c->d_stack_ovf ? c->d_stack_ovf + (size_t)set * ovf_group : nullptr;
        WP.K.ovf_lanes = trace_grid * 256u;
        {
          const std::string e = ovf_layout_error(c, set, trace_grid);
          if (!e.empty()) return fail(c, RT_ERR_STATE, e);
        }
        WP.K.wave_log = debug_passes ? d_wave_log : nullptr;  // COUNT builds (RT_DEBUG_PASSES)
#ifdef RT_DEV
        // RT_DEBUG_WAVES_ONLY: the per-wave timeline without the per-ray step histogram (whose atomics
        // on a few lines would set the pass times)
        if (debug_passes && knob("RT_DEBUG_WAVES_ONLY")) WP.K.flags |= rtd::kFlagNoRayHist;
#endif
        WP.S = c->wfg[set];
        WP.S.pix_xy = c->wf.pix_xy + w0;
        WP.S.pix_acc = c->wf.pix_acc + w0;
        WP.S.cam = cam + w0;
        WP.S.org = org + w0;
        WP.n_frames = f1 - f0;
        WP.pass = 0;
        WP.cam_n = 0u;
        // (not for frame groups of one frame each: their blends must run in frame order)
        WP.fuse_blend = (!pipe && WP.n_frames == 1 && (pix_split || G == 1) && !count) ? 1 : 0;
        slots_g[g] = (unsigned)(f1 - f0) * (w1 - w0);
        // bulk groups (the wf_shade<..., SH_SUB_BULK / CAM> launches) queue the two ray kinds apart
        // (per pass below: passes 1 .. split_passes)
        split_g[g] = (c->split_kinds && c->wide && !count && !c->tile_cost_on && slots_g[g] > c->finish_slots && !WP.fuse_blend) ? 1 : 0;
        sg[g] = pipe ? ps : g == 0 ? c->stream : c->aux[g];
      }
      // camera directions of this call's pixels (every group reads them)
      rtd::WFParams WC = WG[0];
      WC.K.n_work = (unsigned)c->n_valid;
      WC.S.pix_xy = c->wf.pix_xy;
      WC.S.pix_acc = c->wf.pix_acc;
      WC.S.cam = WG[0].S.cam;
      rtd::GroupCounters Z;
      memset(&Z, 0, sizeof(Z));
      Z.n = G;
      for (int g = 0; g < G; g++) Z.cnt[g] = WG[g].S.cnt;
      hipLaunchKernelGGL(rtd::wf_camera, dim3(std::max(1u, std::min<unsigned int>(2048u, ((unsigned)c->n_valid + 255) / 256))),
                         dim3(256), 0, ps, WC, Z);
      HIPCHK(c, hipGetLastError());
      // aux streams start after everything already queued on the caller's stream
      if (G > 1) {
        hipEvent_t es = take_event(c);
        if (!es) return fail(c, RT_ERR_HIP, "hipEventCreate failed");
        HIPCHK(c, hipEventRecord(es, c->stream));
        for (int g = 1; g < G; g++) HIPCHK(c, hipStreamWaitEvent(sg[g], es, 0));
        c->event_pool.push_back(es);  // reusable once the waits are enqueued
      }
      const int last_pass = std::max(0, fp->max_bounce);
      const unsigned int blend_grid = std::max(1u, std::min<unsigned int>(2048u, ((unsigned)c->n_valid + 255) / 256));
      hipEvent_t prev_blend = nullptr;
      for (int g = 0; g < G; g++) {
        rtd::WFParams& WP = WG[g];  // (its pass counters were zeroed by wf_camera)
        // small groups (one frame per call) end their paths in wf_finish after pass finish_pass-1
        int fin_pass = (pipe && c->pipe_finish_pass >= 0) ? c->pipe_finish_pass : c->finish_pass;
#ifdef RT_DEV
        {
          char kn[32];
          snprintf(kn, sizeof(kn), "RT_FINISH_PASS_G%d", g);
          if (const char* e = knob(kn)) fin_pass = std::max(0, atoi(e));
        }
#endif
        const bool finish = !count && !c->tile_cost_on && !(fp->flags & RT_FLAG_NO_FINISH) &&
                            fin_pass >= 1 && fin_pass <= last_pass &&
                            ((fp->flags & RT_FLAG_FINISH) || slots_g[g] <= c->finish_slots);
        // pass 0 queues 16-B rays (WFState::org) unless the finisher takes them over at pass 1
        WP.p1_compact = (finish && fin_pass <= 1) ? 0 : 1;
        for (int pass = 0; pass <= last_pass; pass++) {
          WP.pass = pass;
          WP.split = (split_g[g] && pass >= 1 && pass <= c->split_passes) ? 1 : 0;
          WP.split_out = (split_g[g] && pass + 1 <= c->split_passes) ? 1 : 0;
          if (finish && pass == fin_pass) {
            const dim3 fgrid((unsigned)(c->n_cus * (pipe ? c->pipe_finish_bpc : c->finish_bpc)));
#ifdef RT_DEV
            hipEvent_t ft0 = nullptr, ft1 = nullptr;
            if (debug_passes) {
              HIPCHK(c, hipMemsetAsync(d_wave_log, 0, wave_log.size() * 8, sg[g]));
              ft0 = take_event(c); ft1 = take_event(c);
              HIPCHK(c, hipEventRecord(ft0, sg[g]));
            }
#endif
            if (fp->enable_bsdf) {
              if (c->wide) hipLaunchKernelGGL((rtd::wf_finish<true, true>), fgrid, dim3(256), c->trace_lds, sg[g], WP);
              else hipLaunchKernelGGL((rtd::wf_finish<true, false>), fgrid, dim3(256), c->trace_lds, sg[g], WP);
            } else {
              if (c->wide) hipLaunchKernelGGL((rtd::wf_finish<false, true>), fgrid, dim3(256), c->trace_lds, sg[g], WP);
              else hipLaunchKernelGGL((rtd::wf_finish<false, false>), fgrid, dim3(256), c->trace_lds, sg[g], WP);
            }
            HIPCHK(c, hipGetLastError());
#ifdef RT_DEV
            if (debug_passes) {  // development aid: the finisher's waves (syncs!)
              HIPCHK(c, hipEventRecord(ft1, sg[g]));
              HIPCHK(c, hipStreamSynchronize(sg[g]));
              float ms = 0.0f;
              HIPCHK(c, hipEventElapsedTime(&ms, ft0, ft1));
              c->event_pool.push_back(ft0);
              c->event_pool.push_back(ft1);
              HIPCHK(c, hipMemcpy(wave_log.data(), d_wave_log, wave_log.size() * 8, hipMemcpyDeviceToHost));
              struct FW { double t0, t1, sh_us; unsigned long long it, sh, paths; double at[3]; unsigned long long it_at[3]; };
              std::vector<FW> fw;
              double tmin = 1e300;
              for (size_t w = 0; w < wave_log.size() / 8; w++) {
                const unsigned long long* e = &wave_log[8 * w];
                if (!e[1]) continue;
                FW f{e[0] / 100.0, e[1] / 100.0, e[3] / 100.0, e[2] & 0xfffffull, (e[2] >> 20) & 0xfffffull, e[2] >> 40, {}, {}};
                for (int q = 0; q < 3; q++) {
                  f.at[q] = e[4 + q] ? (double)(e[4 + q] & 0xffffffffull) / 100.0 : -1.0;
                  f.it_at[q] = e[4 + q] >> 32;
                }
                fw.push_back(f);
                tmin = std::min(tmin, e[0] / 100.0);
              }
              std::sort(fw.begin(), fw.end(), [](const FW& a, const FW& b) { return a.t1 > b.t1; });
              unsigned long long paths = 0;
              double life = 0.0, tail16 = 0.0, tail4 = 0.0;
              for (const FW& f : fw) {
                paths += f.paths;
                life += f.t1 - f.t0;
                if (f.at[0] >= 0) tail16 += f.t1 - f.t0 - f.at[0];
                if (f.at[1] >= 0) tail4 += f.t1 - f.t0 - f.at[1];
              }
              fprintf(stderr, "[rt] finisher wave time with <= 16 / <= 4 lanes holding a path (list drained): %.3f / %.3f of %.0f "
                      "wave-us\n", tail16 / std::max(1.0, life), tail4 / std::max(1.0, life), life);
              fprintf(stderr, "[rt] group %d finisher from pass %d: %.3f ms, %zu waves, %llu paths; wave ends (us after the first "
                      "start) 50%% %.1f 90%% %.1f 99%% %.1f 100%% %.1f\n", g, pass, ms, fw.size(), paths,
                      fw.empty() ? 0.0 : fw[fw.size() / 2].t1 - tmin, fw.empty() ? 0.0 : fw[fw.size() / 10].t1 - tmin,
                      fw.empty() ? 0.0 : fw[fw.size() / 100].t1 - tmin, fw.empty() ? 0.0 : fw[0].t1 - tmin);
              for (size_t k = 0; k < std::min<size_t>(6, fw.size()); k++) {
                const FW& f = fw[k];
                fprintf(stderr, "[rt]   wave: start %.1f end %.1f us, %llu paths, %llu trace iterations (%.2f us each outside "
                        "shade), %llu shade steps %.1f us (%.2f us each); <=16 / 4 / 1 busy lanes from %.0f / %.0f / %.0f us "
                        "(iteration %llu / %llu / %llu)\n", f.t0 - tmin, f.t1 - tmin, f.paths, f.it,
                        (f.t1 - f.t0 - f.sh_us) / (double)std::max(1ull, f.it), f.sh, f.sh_us, f.sh_us / (double)std::max(1ull, f.sh),
                        f.at[0], f.at[1], f.at[2], f.it_at[0], f.it_at[1], f.it_at[2]);
              }
            }
#endif
            break;
          }
          // pass 0's camera paths are implicit (wf_trace / wf_shade generate them)
          WP.cam_n = pass == 0 ? slots_g[g] : 0u;
          hipEvent_t t0 = take_event(c), t1 = take_event(c);
          if (!t0 || !t1) return fail(c, RT_ERR_HIP, "hipEventCreate failed");
          HIPCHK(c, hipEventRecord(t0, sg[g]));
          launch_trace(c, count, dim3(pass == 0 ? trace_grid0 : trace_grid1), WP, sg[g], slots_g[g] <= c->finish_slots);
          HIPCHK(c, hipGetLastError());
          HIPCHK(c, hipEventRecord(t1, sg[g]));
          c->trace_events.push_back({t0, t1, c->launches});
          c->trace_launches++;
#ifdef RT_DEV
          if (debug_passes) {  // development aid: per-pass rays / visits / duration (syncs!)
            unsigned long long h[16];
            unsigned int q[8];
            HIPCHK(c, hipStreamSynchronize(sg[g]));
            float ms = 0.0f;
            HIPCHK(c, hipEventElapsedTime(&ms, t0, t1));
            HIPCHK(c, hipMemcpy(h, c->d_stats, sizeof(h), hipMemcpyDeviceToHost));
            HIPCHK(c, hipMemcpy(q, WP.S.cnt, sizeof(q), hipMemcpyDeviceToHost));
            q[0] = q[rtd::cq(pass & 1)] + (WP.split ? q[rtd::cqs(pass & 1)] : 0u);  // (split queues: both kinds)
            fprintf(stderr, "[rt] group %d pass %d: %u rays %.3f ms  cum internal %llu leaf %llu tri %llu iters %llu "
                    "wave-iters max %llu ray-steps max %llu\n", g, pass, (WP.cam_n ? WP.cam_n : q[0]), ms, h[2], h[3], h[4], h[5], h[6], h[7]);
            unsigned long long hq[6];
            HIPCHK(c, hipMemcpy(hq, c->d_stats + 22, sizeof(hq), hipMemcpyDeviceToHost));
            fprintf(stderr, "[rt]   4-wide node visits with BFS index < 1 / 5 / 21 / 64 / 85 / 341: %llu %llu %llu %llu %llu %llu\n",
                    hq[0], hq[1], hq[2], hq[3], hq[4], hq[5]);
            HIPCHK(c, hipMemset(c->d_stats + 22, 0, sizeof(hq)));
            fprintf(stderr, "[rt]   lane utilisation: node phase %.3f (%llu iters)  tri phase %.3f (%llu iters)  busy at "
                    "refill %.3f (%llu outer)\n", h[9] / (64.0 * (double)(h[8] + !h[8])), h[8],
                    h[11] / (64.0 * (double)(h[10] + !h[10])), h[10], h[13] / (64.0 * (double)(h[12] + !h[12])), h[12]);
            fprintf(stderr, "[rt]   overflow-column pushes %llu (%.3f per ray)\n", h[14],
                    (double)h[14] / (double)std::max(1u, WP.cam_n ? WP.cam_n : q[0]));
            HIPCHK(c, hipMemset(c->d_stats + 6, 0, 10 * sizeof(unsigned long long)));
            {  // steps-per-ray histogram (16-step buckets) by ray kind
              unsigned long long hh[64];
              HIPCHK(c, hipMemcpy(hh, c->d_stats + 32, sizeof(hh), hipMemcpyDeviceToHost));
              static const char* kinds[4] = {"cont miss", "cont hit ", "shad miss", "shad hit "};
              for (int kd = 0; kd < 4; kd++) {
                fprintf(stderr, "[rt]   steps/ray %s:", kinds[kd]);
                for (int b = 0; b < 16; b++) fprintf(stderr, " %llu", hh[kd * 16 + b]);
                fprintf(stderr, "\n");
              }
              HIPCHK(c, hipMemset(c->d_stats + 32, 0, sizeof(hh)));
            }
            if (WP.K.wave_log) {
              HIPCHK(c, hipMemcpy(wave_log.data(), d_wave_log, wave_log.size() * 8, hipMemcpyDeviceToHost));
              unsigned long long t0min = ~0ull, t1max = 0, t0max = 0, dmax = 0, itmax = 0, rmax = 0, cmax = 0;
              std::vector<unsigned long long> ends;
              double clk_sum = 0.0, wt_sum = 0.0;
              for (size_t w = 0; w < wave_log.size() / 8; w++) {  // (trace_grid * 4 waves, 4 words each)
                const unsigned long long* e = &wave_log[4 * w];
                const unsigned long long its = e[2] & 0xfffffull, cyc = e[2] >> 20;
                t0min = std::min(t0min, e[0]); t0max = std::max(t0max, e[0]); t1max = std::max(t1max, e[1]);
                if (e[1] - e[0] > dmax) { dmax = e[1] - e[0]; itmax = its; rmax = e[3]; cmax = cyc; }
                if (e[1] > e[0]) { clk_sum += (double)cyc; wt_sum += (double)(e[1] - e[0]); }
                ends.push_back(e[1]);
              }
              fprintf(stderr, "[rt]   shader clock: mean over waves %.0f MHz, longest wave %.0f MHz\n",
                      wt_sum > 0 ? 100.0 * clk_sum / wt_sum : 0.0, dmax ? 100.0 * (double)cmax / (double)dmax : 0.0);
              std::sort(ends.begin(), ends.end());
              auto us = [](unsigned long long t) { return t / 100.0; };  // wall_clock64 = 100 MHz
              fprintf(stderr, "[rt]   waves: start spread %.1f us, span %.1f us; 50%% done at %.1f us, 90%% at %.1f, "
                      "99%% at %.1f; longest wave %.1f us (%llu iters, %llu rays)\n", us(t0max - t0min),
                      us(t1max - t0min), us(ends[ends.size() / 2] - t0min), us(ends[ends.size() * 9 / 10] - t0min),
                      us(ends[ends.size() * 99 / 100] - t0min), us(dmax), itmax, rmax);
            }
          }
#endif
          // (bulk groups: RT_SH_SUB_BULK paths per thread and block-iteration)
          const bool bulk_shade = slots_g[g] > c->finish_slots && !WP.fuse_blend;
          // (the camera pass of a bulk group with >= 64 frames: camera-hit records, wf_shade<..., CAM>)
          const bool cam_shade = RT_CAM_SHADE && bulk_shade && WP.cam_n && WP.n_frames >= 64;
          const unsigned int sub = cam_shade ? (unsigned)rtd::SH_SUB_CAM : bulk_shade ? (unsigned)rtd::SH_SUB_BULK : (unsigned)rtd::SH_SUB;
          const unsigned int shade_grid = std::max(1u, std::min<unsigned int>(4096u, (slots_g[g] + 256u * sub - 1) / (256u * sub)));
          if (fp->enable_bsdf) {
            if (WP.fuse_blend) hipLaunchKernelGGL((rtd::wf_shade<true, true>), dim3(shade_grid), dim3(256), 0, sg[g], WP);
            else if (cam_shade) hipLaunchKernelGGL((rtd::wf_shade<true, false, rtd::SH_SUB_CAM, true>), dim3(shade_grid), dim3(256), 0, sg[g], WP);
            else if (bulk_shade) hipLaunchKernelGGL((rtd::wf_shade<true, false, rtd::SH_SUB_BULK>), dim3(shade_grid), dim3(256), 0, sg[g], WP);
            else hipLaunchKernelGGL((rtd::wf_shade<true, false>), dim3(shade_grid), dim3(256), 0, sg[g], WP);
          } else {
            if (WP.fuse_blend) hipLaunchKernelGGL((rtd::wf_shade<false, true>), dim3(shade_grid), dim3(256), 0, sg[g], WP);
            else if (cam_shade) hipLaunchKernelGGL((rtd::wf_shade<false, false, rtd::SH_SUB_CAM, true>), dim3(shade_grid), dim3(256), 0, sg[g], WP);
            else if (bulk_shade) hipLaunchKernelGGL((rtd::wf_shade<false, false, rtd::SH_SUB_BULK>), dim3(shade_grid), dim3(256), 0, sg[g], WP);
            else hipLaunchKernelGGL((rtd::wf_shade<false, false>), dim3(shade_grid), dim3(256), 0, sg[g], WP);
          }
          HIPCHK(c, hipGetLastError());
        }
        // progressive blend in frame order: group g after group g-1 (pixel groups blend
        // disjoint pixels: no order between them)
        if (prev_blend) {
          HIPCHK(c, hipStreamWaitEvent(sg[g], prev_blend, 0));
          c->event_pool.push_back(prev_blend);
        }
        if (e_entry) {  // pipelined: after the caller's work on the accumulation and the previous call
          HIPCHK(c, hipStreamWaitEvent(sg[g], e_entry, 0));
          c->event_pool.push_back(e_entry);  // reusable once the wait is enqueued
          e_entry = nullptr;
        }
        if (!WP.fuse_blend) {
          hipLaunchKernelGGL(rtd::wf_blend, dim3(blend_grid), dim3(256), 0, sg[g], WP);
          HIPCHK(c, hipGetLastError());
        }
        if (!pix_split && g + 1 < G) {
          prev_blend = take_event(c);
          if (!prev_blend) return fail(c, RT_ERR_HIP, "hipEventCreate failed");
          HIPCHK(c, hipEventRecord(prev_blend, sg[g]));
        }
      }
      // the caller's stream joins the last group (frame groups finish in order through their
      // blends) or every group (pixel groups)
      for (int g = pix_split ? 1 : G - 1; g < G && G > 1; g++) {
        hipEvent_t ej = take_event(c);
        if (!ej) return fail(c, RT_ERR_HIP, "hipEventCreate failed");
        HIPCHK(c, hipEventRecord(ej, sg[g]));
        HIPCHK(c, hipStreamWaitEvent(c->stream, ej, 0));
        c->event_pool.push_back(ej);
      }
    }
    HIPCHK(c, hipEventRecord(e1, ps));
    if (pipe) {  // the caller's stream joins the call; the set is free again after it
      if (c->set_free[pset]) c->event_pool.push_back(c->set_free[pset]);
      c->set_free[pset] = take_event(c);
      if (!c->set_free[pset]) return fail(c, RT_ERR_HIP, "hipEventCreate failed");
      HIPCHK(c, hipEventRecord(c->set_free[pset], ps));
      HIPCHK(c, hipStreamWaitEvent(c->stream, c->set_free[pset], 0));
    } else if (pipe_sets >= 2) {  // pipelined calls that follow start after this batch
      if (!c->batch_done) HIPCHK(c, hipEventCreateWithFlags(&c->batch_done, hipEventDisableTiming));
      HIPCHK(c, hipEventRecord(c->batch_done, c->stream));
    }
    if (!LT->last_use) HIPCHK(c, hipEventCreateWithFlags(&LT->last_use, hipEventDisableTiming));
    HIPCHK(c, hipEventRecord(LT->last_use, c->stream));
    c->events.push_back({e0, e1});
    c->launches++;
    int frc = fold_trace_events(c, kMaxPendingEvents);
    if (!frc) frc = fold_events(c, c->events, c->kernel_ms, kMaxPendingEvents);
    if (frc) return frc;
  }
  return RT_OK;
}

int rt_synchronize(rt_ctx* c) {
  if (!c) return RT_ERR_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  // (the stream joins every group and pipelined set of each call, so all pairs have finished)
  for (auto& e : c->events) {
    const int rc = fold_pair(c, e, c->kernel_ms);
    if (rc) return rc;
  }
  c->events.clear();
  for (auto& e : c->trace_events) {
    const int rc = fold_trace(c, e);
    if (rc) return rc;
  }
  c->trace_events.clear();
  return RT_OK;
}

int rt_abi_version(void) { return RT_ABI_VERSION; }
int rt_gather_last_transport(const rt_ctx* c) { return c ? c->gather_transport : RT_ERR_ARG; }

// rt_stats_get and rt_render write the ABI-3 struct (through p1_rays), the size every binding of
// that header allocated; the fields added since reach a caller only through rt_stats_get_sized
// with its own sizeof(rt_stats)
constexpr size_t kStatsBytesAbi3 = offsetof(rt_stats, pass0_steps);
static_assert(kStatsBytesAbi3 == 13 * 8, "the ABI-3 rt_stats is 13 eight-byte fields");
int stats_fill(rt_ctx* c, rt_stats* st);

int rt_stats_get_sized(rt_ctx* c, rt_stats* st, size_t bytes) {
  if (!c || !st) return RT_ERR_ARG;
  rt_stats full;
  const int rc = stats_fill(c, &full);
  if (rc) return rc;
  memcpy(st, &full, std::min(bytes, sizeof(full)));
  return RT_OK;
}

int rt_stats_get(rt_ctx* c, rt_stats* st) { return rt_stats_get_sized(c, st, kStatsBytesAbi3); }

int stats_fill(rt_ctx* c, rt_stats* st) {
  if (!c || !st) return RT_ERR_ARG;
  int rc = rt_synchronize(c);
  if (rc) return rc;
  memset(st, 0, sizeof(*st));
  std::vector<unsigned long long> all(rtd::kStatWords);
  HIPCHK(c, hipMemcpy(all.data(), c->d_stats, all.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  const unsigned long long* h = all.data();
  unsigned long long shard[3] = {0, 0, 0};  // the per-wave flushes' shard lines (rays, samples, finish steps)
  for (unsigned int s = 0; s < rtd::kStatShards; s++)
    for (int k = 0; k < 3; k++) shard[k] += h[rtd::stats_shard(s) + k];
  st->rays = h[0] + shard[0]; st->samples = h[1] + shard[1];
  st->internal_pops = h[2]; st->leaf_pops = h[3]; st->tri_tests = h[4];
  st->launches = c->launches;
  st->kernel_ms = c->kernel_ms;
  st->trace_launches = c->trace_launches;
  st->trace_ms = c->trace_ms;
  st->trace_iters = h[5];
  st->trace_iters_max = h[6];
  const unsigned long long* ps = h + 16;
  st->path_steps = ps[0];
  st->p1_rays = ps[1];
  st->pass0_steps = ps[2];
  st->pass1_steps = ps[3];
  st->finish_steps = ps[4] + shard[2];
  double busy = c->busy_closed_ms;
  for (const auto& iv : c->busy) busy += iv.hi - iv.lo;
  st->trace_busy_ms = busy;
  return RT_OK;
}

int rt_stats_reset(rt_ctx* c) {
  if (!c) return RT_ERR_ARG;
  int rc = rt_synchronize(c);
  if (rc) return rc;
  HIPCHK(c, hipMemset(c->d_stats, 0, rtd::kStatWords * sizeof(unsigned long long)));
  c->kernel_ms = 0.0;
  c->launches = 0;
  c->trace_ms = 0.0;
  c->trace_launches = 0;
  c->busy.clear();
  c->busy_closed_ms = 0.0;
  return RT_OK;
}

// Per-tile cost probe for a balanced tile assignment (rt_set_tile_owners): renders n_frames with
// the visit-counting trace, which adds every ray's node + triangle steps (+ RT_COST_PER_RAY) to
// its tile's counter.  Integer counts of a deterministic render: the same on every rank and box.
// LoopNum and the accumulation are restored afterwards; the stats counters include the probe.
// One probe render (COUNT build of wf_trace) whose per-ray traversal steps accumulate into n_bins
// costs: per local tile, or per 64-item work block (blocks); accumulation and LoopNum restored.
static int cost_probe(rt_ctx* c, const rt_frame_params* fp, const float* rand_origin, int32_t n_frames, uint64_t* costs,
                      size_t n_bins, bool blocks) {
  int rc = rt_synchronize(c);
  if (rc) return rc;
  HIPCHK(c, hipSetDevice(c->device));
  const size_t abytes = (size_t)std::max(1, c->max_local_tiles) * c->tile_w * c->tile_h * sizeof(float4);
  void* saved = nullptr;
  HIPCHK(c, hipMalloc(&saved, abytes));
  HIPCHK(c, hipMemcpy(saved, c->d_accum, abytes, hipMemcpyDeviceToDevice));
  const int loop = c->loop_num;
  dfree(c->d_tile_cost);
  hipError_t he = hipMalloc(&c->d_tile_cost, n_bins * sizeof(unsigned long long));
  if (he == hipSuccess) he = hipMemset(c->d_tile_cost, 0, n_bins * sizeof(unsigned long long));
  if (he != hipSuccess) {
    (void)hipFree(saved);
    return fail(c, RT_ERR_HIP, std::string("cost probe: ") + hipGetErrorString(he));
  }
  rt_frame_params q = *fp;
  q.flags = (q.flags | RT_FLAG_COUNT_VISITS) & ~RT_FLAG_MEGAKERNEL;
  // rt_order_work ranks blocks by their camera rays alone: the camera pass is the same in every
  // frame (R6), so the order does not depend on the probe frame's random bounces (C3 1080p, 10
  // probe frames: single frames 2.85-2.89 ms with it, 2.85-3.10 ms from whole-path costs)
  if (blocks) q.max_bounce = 0;
  c->tile_cost_on = true;
  c->cost_blocks = blocks;
  rc = rt_render(c, &q, rand_origin, n_frames, nullptr);
  c->tile_cost_on = false;
  c->cost_blocks = false;
  if (rc == RT_OK) {
    he = hipMemcpy(costs, c->d_tile_cost, n_bins * sizeof(uint64_t), hipMemcpyDeviceToHost);
    if (he != hipSuccess) rc = fail(c, RT_ERR_HIP, std::string("cost probe: ") + hipGetErrorString(he));
  } else {
    (void)rt_synchronize(c);  // whatever the failed call queued has finished with the accumulation
  }
  // the accumulation is left as it was, on the error path too (the probe frames may have blended)
  he = hipMemcpy(c->d_accum, saved, abytes, hipMemcpyDeviceToDevice);
  if (he != hipSuccess && rc == RT_OK) rc = fail(c, RT_ERR_HIP, std::string("cost probe: ") + hipGetErrorString(he));
  (void)hipFree(saved);
  dfree(c->d_tile_cost);
  c->loop_num = loop;
  return rc;
}

#ifndef RT_ORDER_HEAD_FRAC
#define RT_ORDER_HEAD_FRAC 0.05
#endif
int rt_order_work(rt_ctx* c, const rt_frame_params* fp, const float* rand_origin, int32_t n_frames) {
  if (!c || !fp || !rand_origin || n_frames <= 0) return RT_ERR_ARG;
  if (!c->frame_set) return fail(c, RT_ERR_STATE, "rt_resize first");
  const size_t nv = (size_t)c->n_valid, nb = nv / 64;  // whole 64-item blocks (a partial one stays last)
  if (nb < 2) return RT_OK;
  std::vector<uint64_t> cost((nv + 63) / 64);
  int rc = cost_probe(c, fp, rand_origin, n_frames, cost.data(), cost.size(), true);
  if (rc) return rc;
  std::vector<uint32_t> sorted(nb), order;
  for (size_t b = 0; b < nb; b++) sorted[b] = (uint32_t)b;
  std::stable_sort(sorted.begin(), sorted.end(), [&](uint32_t a, uint32_t b) { return cost[a] > cost[b]; });
  // the costliest RT_ORDER_HEAD_FRAC of the blocks first: a one-frame call runs them as their own
  // small pixel group beside the rest, so the paths with the longest bounce chains reach their
  // finisher early (C3 1080p: 3.23 -> 3.09 ms synchronised; head 3 / 8 / 12%: -1 / -2.5 / -1.5%;
  // an even split with every group's share dealt round-robin: the round-2 default); the rest
  // follow in descending order, dealt round-robin into the remaining groups' ranges
  int G = std::max(1, c->n_groups);
  double head_frac = G >= 2 ? RT_ORDER_HEAD_FRAC : 0.0;
  if (const char* e = knob("RT_ORDER_RANGES")) G = std::max(1, atoi(e));  // (measurement)
  if (const char* e = knob("RT_ORDER_HEAD")) head_frac = atof(e);         // (measurement)
  order.reserve(nb);
  const size_t head = std::min(nb, (size_t)((double)nb * std::max(0.0, head_frac)));
  for (size_t k = 0; k < head; k++) order.push_back(sorted[k]);
  if (head > 0) G = std::max(1, G - 1);
  for (int g = 0; g < G; g++)
    for (size_t k = head + (size_t)g; k < nb; k += (size_t)G) order.push_back(sorted[k]);
  c->order_head = head * 64;
  // permute the pixel list (xy then accumulation index) by whole blocks: a wave keeps its 8x8
  // block, and the blocks whose rays cost most are queued (and claimed) first
  std::vector<unsigned int> pix(2 * nv), out(2 * nv);
  HIPCHK(c, hipMemcpy(pix.data(), c->d_pix, 2 * nv * sizeof(unsigned int), hipMemcpyDeviceToHost));
  for (size_t k = 0; k < nb; k++)
    for (size_t j = 0; j < 64; j++) {
      out[k * 64 + j] = pix[(size_t)order[k] * 64 + j];
      out[nv + k * 64 + j] = pix[nv + (size_t)order[k] * 64 + j];
    }
  for (size_t j = nb * 64; j < nv; j++) {
    out[j] = pix[j];
    out[nv + j] = pix[nv + j];
  }
  HIPCHK(c, hipMemcpy(c->d_pix, out.data(), 2 * nv * sizeof(unsigned int), hipMemcpyHostToDevice));
  return RT_OK;
}

int rt_tile_costs(rt_ctx* c, const rt_frame_params* fp, const float* rand_origin, int32_t n_frames, uint64_t* costs) {
  if (!c || !fp || !rand_origin || !costs || n_frames <= 0) return RT_ERR_ARG;
  if (!c->frame_set) return fail(c, RT_ERR_STATE, "rt_resize first");
  if (c->local_tiles == 0) return RT_OK;
  return cost_probe(c, fp, rand_origin, n_frames, costs, (size_t)c->local_tiles, false);
}

int rt_render(rt_ctx* c, const rt_frame_params* fp, const float* rand_origin, int32_t n_frames, rt_stats* st) {
  int rc = rt_render_async(c, fp, rand_origin, n_frames);
  if (rc) return rc;
  return st ? rt_stats_get(c, st) : rt_synchronize(c);
}

// the display pass into c->d_disp on the ctx stream (after every render call queued before it)
static int display_kernel(rt_ctx* c, const float* frame_device, int32_t flags) {
  if (!c->frame_set) return fail(c, RT_ERR_STATE, "resize first");
  if (!frame_device && c->world != 1)
    return fail(c, RT_ERR_STATE, "a multi-rank context displays an assembled frame (rt_assemble_frame)");
  HIPCHK(c, hipSetDevice(c->device));
  const size_t bytes = (size_t)c->W * c->H * 3;
  if (bytes > c->disp_bytes) {
    HIPCHK(c, hipStreamSynchronize(c->stream));  // an earlier display may still read it
    dfree(c->d_disp);
    HIPCHK(c, hipMalloc(&c->d_disp, bytes));
    c->disp_bytes = bytes;
  }
  dim3 grid((c->W + 255) / 256, c->H);
  hipLaunchKernelGGL(rtd::rt_display_kernel, grid, dim3(256), 0, c->stream,
                     frame_device ? nullptr : c->d_accum, frame_device, (unsigned char*)c->d_disp, c->W, c->H,
                     c->tile_w, c->tile_h, c->tiles_x, (int)flags);
  HIPCHK(c, hipGetLastError());
  return RT_OK;
}

int rt_tonemap(rt_ctx* c, const float* frame_device, int32_t flags, uint8_t* rgb8_host) {
  if (!c || !rgb8_host) return RT_ERR_ARG;
  if (int rc = display_kernel(c, frame_device, flags)) return rc;
  HIPCHK(c, hipMemcpyAsync(rgb8_host, c->d_disp, (size_t)c->W * c->H * 3, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return RT_OK;
}

int rt_tonemap_async(rt_ctx* c, const float* frame_device, int32_t flags, int32_t slot) {
  if (!c || slot < 0 || slot >= rt_ctx::DISP_SLOTS) return RT_ERR_ARG;
  rt_ctx::DisplaySlot& d = c->disp[slot];
  if (d.ev) HIPCHK(c, hipEventSynchronize(d.ev));  // the slot's previous image has been copied out
  if (int rc = display_kernel(c, frame_device, flags)) return rc;
  const size_t bytes = (size_t)c->W * c->H * 3;
  if (bytes > d.cap) {
    if (d.host) (void)hipHostFree(d.host);
    d.host = nullptr;
    d.cap = 0;
    HIPCHK(c, hipHostMalloc((void**)&d.host, bytes));
    d.cap = bytes;
  }
  if (!d.ev) HIPCHK(c, hipEventCreateWithFlags(&d.ev, hipEventDisableTiming));
  HIPCHK(c, hipMemcpyAsync(d.host, c->d_disp, bytes, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipEventRecord(d.ev, c->stream));
  d.bytes = bytes;
  return RT_OK;
}

int rt_display_fetch(rt_ctx* c, int32_t slot, uint8_t* rgb8_host) {
  if (!c || !rgb8_host || slot < 0 || slot >= rt_ctx::DISP_SLOTS) return RT_ERR_ARG;
  rt_ctx::DisplaySlot& d = c->disp[slot];
  if (!d.ev || !d.bytes) return fail(c, RT_ERR_STATE, "rt_display_fetch: nothing displayed into this slot");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipEventSynchronize(d.ev));
  memcpy(rgb8_host, d.host, d.bytes);
  return RT_OK;
}

int rt_get_stream(const rt_ctx* c, void** stream) {
  if (!c || !stream) return RT_ERR_ARG;
  *stream = (void*)c->stream;
  return RT_OK;
}

int rt_set_stream(rt_ctx* c, void* stream) {
  if (!c) return RT_ERR_ARG;
  int rc = rt_synchronize(c);
  if (rc) return rc;
  if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
  if (stream) {
    c->stream = (hipStream_t)stream;
    c->own_stream = false;
  } else {
    HIPCHK(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    c->own_stream = true;
  }
  return RT_OK;
}

static int accum_transfer(rt_ctx* c, float* host, int32_t layout, bool to_host) {
  if (!c || !host || (layout != RT_LAYOUT_FRAME && layout != RT_LAYOUT_LOCAL_TILES)) return RT_ERR_ARG;
  if (!c->frame_set) return fail(c, RT_ERR_STATE, "rt_resize first");
  int rc = rt_synchronize(c);
  if (rc) return rc;
  const size_t tpx = (size_t)c->tile_w * c->tile_h;
  std::vector<float4> buf((size_t)std::max(1, c->max_local_tiles) * tpx);
  HIPCHK(c, hipMemcpy(buf.data(), c->d_accum, buf.size() * sizeof(float4), hipMemcpyDeviceToHost));
  for (int lt = 0; lt < c->local_tiles; lt++) {
    int gt = c->my_tiles[lt];
    int tx = gt % c->tiles_x, ty = gt / c->tiles_x;
    for (int ly = 0; ly < c->tile_h; ly++)
      for (int lx = 0; lx < c->tile_w; lx++) {
        size_t li = (size_t)lt * tpx + (size_t)ly * c->tile_w + lx;
        float* h;
        if (layout == RT_LAYOUT_LOCAL_TILES) {
          h = host + 3 * li;
        } else {
          int px = tx * c->tile_w + lx, py = ty * c->tile_h + ly;
          if (px >= c->W || py >= c->H) continue;
          h = host + 3 * ((size_t)py * c->W + px);
        }
        if (to_host) { h[0] = buf[li].x; h[1] = buf[li].y; h[2] = buf[li].z; }
        else buf[li] = make_float4(h[0], h[1], h[2], 0.0f);
      }
  }
  if (!to_host) HIPCHK(c, hipMemcpy(c->d_accum, buf.data(), buf.size() * sizeof(float4), hipMemcpyHostToDevice));
  return RT_OK;
}

int rt_read_accum(rt_ctx* c, float* rgb_out, int32_t layout) { return accum_transfer(c, rgb_out, layout, true); }
int rt_write_accum(rt_ctx* c, const float* rgb_in, int32_t layout) {
  return accum_transfer(c, const_cast<float*>(rgb_in), layout, false);
}

int rt_accum_device(const rt_ctx* c, void** ptr, size_t* bytes, int32_t* local_tiles, int32_t* max_local_tiles) {
  if (!c || !ptr || !bytes) return RT_ERR_ARG;
  if (!c->frame_set) return RT_ERR_STATE;
  *ptr = c->d_accum;
  *bytes = (size_t)std::max(1, c->max_local_tiles) * c->tile_w * c->tile_h * sizeof(float4);
  if (local_tiles) *local_tiles = c->local_tiles;
  if (max_local_tiles) *max_local_tiles = c->max_local_tiles;
  return RT_OK;
}

int rt_copy_accum_device(rt_ctx* c, void* dst, size_t bytes) {
  if (!c || !dst) return RT_ERR_ARG;
  if (!c->frame_set) return fail(c, RT_ERR_STATE, "rt_resize first");
  size_t have = (size_t)std::max(1, c->max_local_tiles) * c->tile_w * c->tile_h * sizeof(float4);
  if (bytes > have) return fail(c, RT_ERR_ARG, "copy larger than the accumulation buffer");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipMemcpyAsync(dst, c->d_accum, bytes, hipMemcpyDeviceToDevice, c->stream));
  return RT_OK;
}

int rt_assemble_frame(rt_ctx* c, const void* gathered, int32_t world, void* frame) {
  if (!c || !gathered || !frame || world <= 0) return RT_ERR_ARG;
  if (!c->frame_set) return fail(c, RT_ERR_STATE, "rt_resize first");
  if (world != c->world) return fail(c, RT_ERR_ARG, "world differs from the tiling");
  HIPCHK(c, hipSetDevice(c->device));
  dim3 block(256), grid((c->W + 255) / 256, c->H);
  hipLaunchKernelGGL(rtd::rt_assemble_kernel, grid, block, 0, c->stream, (const float4*)gathered, (float*)frame, c->W,
                     c->H, c->tile_w, c->tile_h, c->tiles_x, (const int2*)c->d_tile_src, std::max(1, c->max_local_tiles));
  HIPCHK(c, hipGetLastError());
  return RT_OK;
}

int rt_gather(rt_ctx* const* ctxs, int32_t n, float* full_rgb) {
  return rt_gather_ex(ctxs, n, full_rgb, RT_GATHER_AUTO);
}

// RCCL form of the gather: one communicator per context's device (ncclCommInitAll,
// this thread drives every rank), each rank's tiles sent to rank 0 on its own stream after its
// queued work, rank 0 receiving all of them (its own included) into the rank-major buffer, in one
// group.  The communicators stay in ctxs[0] for the next gather over the same devices.
static int gather_rccl(rt_ctx* const* ctxs, int n, char* g, size_t part) {
  rt_ctx* c0 = ctxs[0];
  std::vector<int> devs(n);
  for (int r = 0; r < n; r++) devs[r] = ctxs[r]->device;
  auto nfail = [&](const char* what, ncclResult_t e) {
    return fail(c0, RT_ERR_HIP, std::string("rt_gather: ") + what + ": " + ncclGetErrorString(e));
  };
  if (c0->rccl_devs != devs) {
    for (auto& m : c0->rccl_comms) (void)ncclCommDestroy(m);
    c0->rccl_comms.assign(n, nullptr);
    c0->rccl_devs.clear();
    const ncclResult_t e = ncclCommInitAll(c0->rccl_comms.data(), n, devs.data());
    if (e != ncclSuccess) {
      c0->rccl_comms.clear();
      return nfail("ncclCommInitAll", e);
    }
    c0->rccl_devs = devs;
  }
  const size_t cnt = part / sizeof(float);
  ncclResult_t e = ncclGroupStart();
  if (e != ncclSuccess) return nfail("ncclGroupStart", e);
  for (int r = 0; r < n && e == ncclSuccess; r++) {
    (void)hipSetDevice(ctxs[r]->device);
    e = ncclSend(ctxs[r]->d_accum, cnt, ncclFloat32, 0, c0->rccl_comms[r], ctxs[r]->stream);
  }
  (void)hipSetDevice(c0->device);
  for (int r = 0; r < n && e == ncclSuccess; r++)
    e = ncclRecv(g + (size_t)r * part, cnt, ncclFloat32, r, c0->rccl_comms[0], c0->stream);
  const ncclResult_t eg = ncclGroupEnd();
  (void)hipSetDevice(c0->device);
  if (e != ncclSuccess) return nfail("ncclSend / ncclRecv", e);
  if (eg != ncclSuccess) return nfail("ncclGroupEnd", eg);
  return RT_OK;
}

int rt_gather_ex(rt_ctx* const* ctxs, int32_t n, float* full_rgb, int32_t transport) {
  if (!ctxs || n <= 0 || !full_rgb || !ctxs[0]) return RT_ERR_ARG;
  if (transport != RT_GATHER_AUTO && transport != RT_GATHER_RCCL && transport != RT_GATHER_PEER) return RT_ERR_ARG;
  rt_ctx* c0 = ctxs[0];
  for (int r = 0; r < n; r++) {
    const rt_ctx* c = ctxs[r];
    if (!c) return fail(c0, RT_ERR_ARG, "rt_gather: null context");
    if (!c->frame_set) return fail(c0, RT_ERR_STATE, "rt_gather: rt_resize every context first");
    if (c->rank != r || c->world != n) return fail(c0, RT_ERR_ARG, "rt_gather: ctxs[r] must render rank r of a world of n");
    if (c->W != c0->W || c->H != c0->H || c->tile_w != c0->tile_w || c->tile_h != c0->tile_h ||
        c->max_local_tiles != c0->max_local_tiles || c->owner != c0->owner)
      return fail(c0, RT_ERR_ARG, "rt_gather: contexts differ in frame size or tiling");
  }
  bool distinct = true;  // one device per context: what an RCCL communicator needs
  for (int r = 0; r < n; r++)
    for (int q = 0; q < r; q++) distinct &= ctxs[r]->device != ctxs[q]->device;
  if (transport == RT_GATHER_AUTO) transport = distinct ? RT_GATHER_RCCL : RT_GATHER_PEER;
  if (transport == RT_GATHER_RCCL && !distinct)
    return fail(c0, RT_ERR_ARG, "rt_gather: RCCL needs one device per context (use RT_GATHER_PEER)");
  const size_t part = (size_t)std::max(1, c0->max_local_tiles) * c0->tile_w * c0->tile_h * sizeof(float4);
  const size_t frame = (size_t)c0->W * c0->H * 3 * sizeof(float);
  HIPCHK(c0, hipSetDevice(c0->device));
  if (part * n + frame > c0->gather_bytes) {
    dfree(c0->d_gather);
    c0->gather_bytes = 0;
    HIPCHK(c0, hipMalloc(&c0->d_gather, part * n + frame));
    c0->gather_bytes = part * n + frame;
  }
  char* g = static_cast<char*>(c0->d_gather);
  std::vector<std::pair<int, hipEvent_t>> done;  // (device, event) per rank, destroyed after the copy
  auto cleanup = [&]() {
    for (auto& e : done) { (void)hipSetDevice(e.first); (void)hipEventDestroy(e.second); }
    (void)hipSetDevice(c0->device);
  };
  int rc = RT_OK;
  c0->gather_transport = transport;
  if (transport == RT_GATHER_RCCL) rc = gather_rccl(ctxs, n, g, part);
  for (int r = 0; r < n && rc == RT_OK && transport == RT_GATHER_PEER; r++) {
    const rt_ctx* c = ctxs[r];
    hipEvent_t e = nullptr;
    hipError_t he = hipSetDevice(c->device);
    if (he == hipSuccess) he = hipEventCreateWithFlags(&e, hipEventDisableTiming);
    if (he == hipSuccess) done.push_back({c->device, e});
    if (he == hipSuccess) he = hipEventRecord(e, c->stream);  // after everything queued on rank r
    if (he == hipSuccess) he = hipSetDevice(c0->device);
    if (he == hipSuccess && c->device != c0->device) {  // direct xGMI copies where the link allows
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, c0->device, c->device) == hipSuccess && can) {
        const hipError_t pe = hipDeviceEnablePeerAccess(c->device, 0);
        if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled) he = pe;
        (void)hipGetLastError();
      }
    }
    if (he == hipSuccess) he = hipStreamWaitEvent(c0->stream, e, 0);
    if (he == hipSuccess)
      he = hipMemcpyPeerAsync(g + (size_t)r * part, c0->device, c->d_accum, c->device, part, c0->stream);
    if (he != hipSuccess) rc = fail(c0, RT_ERR_HIP, std::string("rt_gather: ") + hipGetErrorString(he));
  }
  if (rc == RT_OK) rc = rt_assemble_frame(c0, g, n, g + (size_t)n * part);
  if (rc == RT_OK) {
    hipError_t he = hipMemcpyAsync(full_rgb, g + (size_t)n * part, frame, hipMemcpyDeviceToHost, c0->stream);
    if (he == hipSuccess) he = hipStreamSynchronize(c0->stream);
    if (he != hipSuccess) rc = fail(c0, RT_ERR_HIP, std::string("rt_gather: ") + hipGetErrorString(he));
  } else {
    (void)hipStreamSynchronize(c0->stream);  // the events may still be waited on
  }
  cleanup();
  return rc;
}

}  // extern "C"
