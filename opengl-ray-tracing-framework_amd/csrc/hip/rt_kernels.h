// rt_kernels.h — the persistent-thread path-tracing megakernel for gfx950.
//
// One lane = one pixel path (the reference's one fragment invocation, RT:1518-1558), but
// restructured for a 64-wide wavefront:
//   * persistent grid sized to residency; lanes pull pixels from a global work counter with
//     one wave-aggregated atomic (ballot + popcount), so a lane whose path ended starts the
//     next pixel/frame immediately (path regeneration) instead of idling to the wave's
//     longest path;
//   * the bounce loop of shadingImportanceSampling_BSDF (RT:1369-1516) is unrolled into a
//     per-lane state machine with ONE traversal site: camera, NEE-shadow and continuation
//     rays of different lanes traverse the BVH together in the same loop;
//   * traversal = the reference's near-first stack order (RT:338-392) with the stack in LDS
//     ([entry][lane] layout, conflict-free), child boxes stored in the parent node (one 64-B
//     fetch per internal node), leaves referenced by triangle range (no leaf fetch),
//     closest-hit culling of popped subtrees (R2 notes the reference visits every hit box;
//     culling never changes the closest hit) and any-hit termination for shadow rays (only
//     isHit is consumed, RT:1389);
//   * triangles as 3 x float4 {p, Ng} with the geometric normal precomputed by the same
//     fp32 ops the shader performs per test (RT:253); normals/material fetched once per
//     closest hit instead of on every closer hit (RT:330).
// Arithmetic on every value that reaches the image follows the shader's evaluation order.
#pragma once
#include "rt_device.h"
#include "rt_abi.h"

namespace rtd {

enum : int { PH_IDLE = 0, PH_START = 1, PH_CAMERA = 2, PH_SHADOW = 3, PH_CONT = 4 };

struct KParams {
  float pos[3], lbc[3], right[3], up[3];
  float half_w, half_h;
  int enable_mis, enable_env, enable_bsdf;
  float env_intensity, env_angle;
  int max_bounce, flags, n_frames;
  const int* __restrict__ loop_num;       // per frame of this launch (device table)
  const float* __restrict__ rand_origin;  // per frame of this launch (device table)
  const float2* __restrict__ sobol;       // per frame of this launch: sobolVec2 of bounces 0..3 (wf_sobol)
  const float2* __restrict__ blend_w;     // per frame of this launch: blend weights {1/n, (n-1)/n} (wf_sobol)
  int W, H, tile_w, tile_h, tiles_x, rank, world;
  const int* __restrict__ tile_ids;   // global tile id of each local tile (rt_set_tile_owners)
  unsigned long long* __restrict__ tile_cost;  // rt_tile_costs probe: per local tile (else null)
  int cost_blocks;                  // tile_cost indexed by 64-item work block (rt_order_work) instead of tile
  unsigned int n_work;
  const GNode* __restrict__ nodes;  // binary tree; GNode.ref.z = DFS rank of the first leaf on the right
  int root, has_scene, stack_entries;
  const QNode* __restrict__ qnodes;  // 4-wide collapse of `nodes` (wavefront trace, TW_WIDE)
  int qroot;
  int n_qnodes, n_tri;              // (bounds of the RT_CHECK development build)
  int lds_entries;                  // wavefront traversal: stack entries kept in LDS
  int stack_cap;                    // the deepest stack of the scene's trees (a lane-quad move copies up to it)
  float cull_eps;                   // culling bound: accepted hit points lie within this of their box
  int pool_chunk;                   // wavefront traversal: rays claimed per queue atomic
  int2* __restrict__ stack_ovf;     // deeper entries: [entry - lds_entries][grid lane]
  unsigned int ovf_lanes;
  const float4* __restrict__ tri;   // 3 per triangle: {p1, Ng.x} {p2, Ng.y} {p3, Ng.z}
  const float4* __restrict__ trx;   // traversal record, 3 per triangle: {p1, Ng.x} {R2, Ng.y} {R3, Ng.z}
  float tri_k1, tri_k0;             // its edge-filter margin (csrc/common/tri_filter.h)
  const float4* __restrict__ trin;  // 3 per triangle: {n1, matid bits} {n2, leaf rank bits} {n3, 0}
  const float4* __restrict__ hrec;  // 8 per triangle (one 128-B line): tri's 3 then trin's 3, 2 unused
  const float4* __restrict__ mats;  // 8 per material
  const float4* __restrict__ hdr;
  const float2* __restrict__ cache;  // hdrCache.rg (hdr.w holds hdrCache.b)
  const float4* __restrict__ light;  // NEE light samples per hdrCache texel (SampleHdrLight)
  int hdr_w, hdr_h, hdr_res;
  float4* __restrict__ accum;
  unsigned int* __restrict__ counter;
  unsigned long long* __restrict__ stats;  // rays, samples, internal, leaf, tri
  unsigned long long* __restrict__ wave_log;  // debug (RT_DEBUG_PASSES): per trace wave {t0, t1, iters, rays}
};

struct Visits {
  unsigned long long internal, leaf, tri;
};

// hitAABB RT:303-316.  Returns the reference's distance (entry t0, or exit t1 when the origin
// is inside the box; -1 on a miss) and the entry distance t0 used for culling: a box that
// contains the origin (t0 <= 0) must never be culled.
RTD float slab(f3 o, f3 inv, f3 AA, f3 BB, float& t0_out) {
  f3 f = (BB - o) * inv;
  f3 n = (AA - o) * inv;
  float tmaxx = max_(f.x, n.x), tmaxy = max_(f.y, n.y), tmaxz = max_(f.z, n.z);
  float tminx = min_(f.x, n.x), tminy = min_(f.y, n.y), tminz = min_(f.z, n.z);
  float t1 = min_(tmaxx, min_(tmaxy, tmaxz));
  float t0 = max_(tminx, max_(tminy, tminz));
  t0_out = t0;
  return (t1 >= t0) ? ((t0 > 0.0f) ? t0 : t1) : -1.0f;
}

// Culling bound: a popped subtree whose box entry lies beyond this can hold no hit the reference
// would accept at dist <= best.  Accepted hit points lie within P.cull_eps of their triangle's
// boxes (cull_bound_stats in rt_render.hip), so a triangle's t is at least t0 - cull_eps *
// max|1/d_a|; the 1e-3 terms cover the relative rounding of t0, t and dist = t - 1e-5.  A ray with
// a zero direction component (1/d infinite) is never culled.
RTD float cull_limit(float best, float eps, float ix, float iy, float iz) {
  const float m = fmaxf(fabsf(ix), fmaxf(fabsf(iy), fabsf(iz)));
  return best + 1e-3f + best * 1e-3f + eps * m;
}

template <bool COUNT>
RTD void trace(const KParams& P, f3 o, f3 d, bool anyhit, bool cull, int* __restrict__ sref,
               float* __restrict__ sdist, int stride, int& besttri, float& bestt, Visits& vis) {
  besttri = -1;
  bestt = 0.0f;
  if (!P.has_scene) return;
  f3 inv = mk3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  float best = INF;
  int sp = 0;
  int cur = P.root;
  while (true) {
    bool descend = false;
    if (ref_is_leaf(cur)) {
      if (COUNT) vis.leaf++;
      int first = leaf_first(cur);
      int last = first + leaf_count(cur);
      bool done = false;
      for (int i = first; i < last; ++i) {
        if (COUNT) vis.tri++;
        float4 A = P.tri[3 * i], B = P.tri[3 * i + 1], Cc = P.tri[3 * i + 2];
        f3 p1 = xyz(A), p2 = xyz(B), p3 = xyz(Cc);
        f3 ng = mk3(A.w, B.w, Cc.w);
        float dn = dot(ng, d);
        if (fabs_(dn) < 0.00001f) continue;                       // RT:262
        float t = (dot(ng, p1) - dot(o, ng)) / dot(d, ng);        // RT:265
        if (!(t >= 0.0005f)) continue;                            // RT:268
        float dist = t - 0.00001f;                                // RT:284
        if (!(dist < best)) continue;                             // RT:328, RT:356
        f3 Pp = o + d * t;
        float e1 = dot(cross(p2 - p1, Pp - p1), ng);
        float e2 = dot(cross(p3 - p2, Pp - p2), ng);
        float e3 = dot(cross(p1 - p3, Pp - p3), ng);
        if ((e1 > 0 && e2 > 0 && e3 > 0) || (e1 < 0 && e2 < 0 && e3 < 0)) {  // RT:278-281
          best = dist;
          besttri = i;
          bestt = t;
          if (anyhit) { done = true; break; }
        }
      }
      if (done) break;
    } else {
      if (COUNT) vis.internal++;
      const GNode nd = P.nodes[cur];
      float e1, e2;  // entry distances (culling keys)
      float d1 = slab(o, inv, mk3(nd.b0.x, nd.b0.y, nd.b0.z), mk3(nd.b0.w, nd.b1.x, nd.b1.y), e1);
      float d2 = slab(o, inv, mk3(nd.b1.z, nd.b1.w, nd.b2.x), mk3(nd.b2.y, nd.b2.z, nd.b2.w), e2);
      // RT:373-388: push far, pop near (equivalently: descend into near, stack the far one)
      int nearRef = 0;
      float nearD = 0.0f;
      if (d1 > 0 && d2 > 0) {
        bool leftFirst = d1 < d2;
        nearRef = leftFirst ? nd.ref.x : nd.ref.y;
        nearD = leftFirst ? e1 : e2;
        sref[sp * stride] = leftFirst ? nd.ref.y : nd.ref.x;
        sdist[sp * stride] = leftFirst ? e2 : e1;
        ++sp;
        descend = true;
      } else if (d1 > 0) {
        nearRef = nd.ref.x; nearD = e1; descend = true;
      } else if (d2 > 0) {
        nearRef = nd.ref.y; nearD = e2; descend = true;
      }
      if (descend && cull && nearD > cull_limit(best, P.cull_eps, inv.x, inv.y, inv.z)) descend = false;
      if (descend) { cur = nearRef; continue; }
    }
    // pop (RT:348), skipping subtrees that start beyond the current closest hit
    bool found = false;
    while (sp > 0) {
      --sp;
      int r = sref[sp * stride];
      float dd = sdist[sp * stride];
      if (cull && dd > cull_limit(best, P.cull_eps, inv.x, inv.y, inv.z)) continue;
      cur = r;
      found = true;
      break;
    }
    if (!found) break;
  }
}

template <bool COUNT>
__global__ __launch_bounds__(256) void rt_path_kernel(const KParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int stride = blockDim.x;
  int* sref = reinterpret_cast<int*>(smem) + threadIdx.x;
  float* sdist = reinterpret_cast<float*>(smem + (size_t)P.stack_entries * stride * 4) + threadIdx.x;
  const Env E{P.hdr, P.cache, P.light, P.hdr_w, P.hdr_h, P.hdr_res, P.env_angle, P.env_intensity};
  const bool cull = (P.flags & RT_FLAG_NO_CULL) == 0;
  const int lane = (int)(threadIdx.x & 63);
  const f3 camPos = mk3(P.pos[0], P.pos[1], P.pos[2]);
  const int tpx = P.tile_w * P.tile_h;

  int phase = PH_IDLE, frame = 0, bounce = 0, mat = 0, accIdx = 0;
  bool exhausted = false, medS = false;
  float u = 0.0f, v = 0.0f, hDist = 0.0f, evp = 0.0f;
  uint32_t wseed = 0;
  f3 acc = splat(0.0f), Le0 = splat(0.0f), Lo = splat(0.0f), hist = splat(1.0f);
  f3 hP = splat(0.0f), hN = splat(0.0f), hV = splat(0.0f), evf = splat(0.0f);
  f3 ro = splat(0.0f), rd = splat(0.0f);
  int trTri = -1;
  float trT = 0.0f;
  unsigned long long nrays = 0, nsamples = 0;
  Visits vis{0, 0, 0};

  while (true) {
    // ------------------------------------------------ consume the last traversal result
    bool doBounce = false, doSample = false, doFinish = false;
    f3 fin = splat(0.0f);
    if (phase == PH_CAMERA || phase == PH_CONT) {
      if (trTri >= 0) {
        // HitRecord of the closest triangle (RT:282-295)
        float4 A = P.tri[3 * trTri], B = P.tri[3 * trTri + 1], Cc = P.tri[3 * trTri + 2];
        float4 N1 = P.trin[3 * trTri], N2 = P.trin[3 * trTri + 1], N3 = P.trin[3 * trTri + 2];
        f3 p1 = xyz(A), p2 = xyz(B), p3 = xyz(Cc);
        f3 ng = mk3(A.w, B.w, Cc.w);
        bool inside = dot(ng, rd) > 0.0f;
        f3 Pp = ro + rd * trT;
        float alpha = (-(Pp.x - p2.x) * (p3.y - p2.y) + (Pp.y - p2.y) * (p3.x - p2.x)) /
                      (-(p1.x - p2.x) * (p3.y - p2.y) + (p1.y - p2.y) * (p3.x - p2.x) + 1e-7f);
        float beta = (-(Pp.x - p3.x) * (p1.y - p3.y) + (Pp.y - p3.y) * (p1.x - p3.x)) /
                     (-(p2.x - p3.x) * (p1.y - p3.y) + (p2.y - p3.y) * (p1.x - p3.x) + 1e-7f);
        float gama = 1.0f - alpha - beta;
        f3 Ns = normalize(alpha * xyz(N1) + beta * xyz(N2) + gama * xyz(N3));
        int nmat = __float_as_int(N1.w);
        if (phase == PH_CONT) {  // RT:1509-1510 emissive of the next hit
          f3 Le = xyz(P.mats[8 * nmat]);
          Lo = Lo + hist * Le * evf / evp;
          bounce++;
        } else {  // RT:1541-1544 first hit
          Le0 = xyz(P.mats[8 * nmat]);
          Lo = splat(0.0f);
          hist = splat(1.0f);
          bounce = 0;
        }
        hP = Pp;
        hN = inside ? -Ns : Ns;
        hV = rd;
        hDist = trT - 0.00001f;
        mat = nmat;
        if (bounce < P.max_bounce) doBounce = true;
        else { fin = Le0 + Lo; doFinish = true; }
      } else if (phase == PH_CAMERA) {  // RT:1532-1539
        fin = P.enable_env ? hdrColor(E, rd) * E.intensity : getDefaultSkyColor(rd.y);
        doFinish = true;
      } else {  // continuation ray escaped (RT:1483-1506)
        if (P.enable_env) {
          f3 light_fr;
          float light_pdf;
          hdrColorPdf(E, rd, light_fr, light_pdf);
          light_fr = light_fr * E.intensity;
          float mis_weight = misMixWeight(evp, light_pdf);
          if (!P.enable_mis) mis_weight = 1.0f;
          if (!medS) Lo = Lo + mis_weight * hist * light_fr * evf / evp;
          else Lo = Lo + hist * light_fr * evf / light_pdf;
        } else {
          f3 light_fr = getDefaultSkyColor(rd.y);
          Lo = Lo + hist * light_fr * evf / evp;
        }
        fin = Le0 + Lo;
        doFinish = true;
      }
    } else if (phase == PH_SHADOW) {
      if (trTri < 0) {  // NEE to the environment (RT:1389-1405)
        const Mat m = load_mat(P.mats, mat);
        f3 L = rd;
        f3 light_fr;
        float light_pdf;
        hdrColorPdf(E, L, light_fr, light_pdf);
        light_fr = light_fr * E.intensity;
        float disney_eval_pdf;
        f3 disney_eval_fr = DisneyEval(m, -hV, hN, L, disney_eval_pdf);
        float mis_weight = misMixWeight(light_pdf, disney_eval_pdf);
        if (!P.enable_mis) mis_weight = 1.0f;
        Lo = Lo + mis_weight * hist * light_fr * disney_eval_fr / light_pdf;
      }
      doSample = true;
    }

    // -------------------------------------------------- bounce start: NEE light sample
    if (doBounce) {
      float xa = rand_(wseed);  // R24
      float xb = rand_(wseed);
      f3 L = SampleHdr(E, xa, xb);
      if (dot(hN, L) > 0.0f) {
        ro = hP;
        rd = L;
        phase = PH_SHADOW;
      } else {
        doSample = true;
      }
    }

    // --------------------------------------------- BSDF sample + continuation ray setup
    if (doSample) {
      const Mat m = load_mat(P.mats, mat);
      f3 V = -hV;
      int g = (P.loop_num[frame] + 1);
      g = g ^ (g >> 1);  // grayCode RT:598
      float sx = sobol_gray(bounce * 2, g);
      float sy = sobol_gray(bounce * 2 + 1, g);
      float cu = rand_(wseed), cv = rand_(wseed);  // CranleyPattersonRotation RT:772-785
      sx += cu;
      if (sx > 1) sx -= 1;
      if (sx < 0) sx += 1;
      sy += cv;
      if (sy > 1) sy -= 1;
      if (sy < 0) sy += 1;
      float xi_3 = rand_(wseed);
      f3 L;
      float pdf;
      bool isRefract;
      f3 fr = DisneySample(sx, sy, xi_3, m, V, hN, L, pdf, isRefract);
      medS = false;
      float scatter_pdf = 0.0f;
      float transmittance = 1.0f;
      if (pdf > 0.0f) {
        if (!isRefract) {
          hist = hist * (fr / pdf);
        } else if (m.mtype == MEDIUM_ABSORB) {
          hist = hist * exp3(-(splat(1.0f) - m.mcolor) * hDist * m.mdensity);
        } else if (m.mtype == MEDIUM_EMISSIVE) {
          Lo = Lo + m.mcolor * hDist * m.mdensity * hist;
        } else if (m.mtype == MEDIUM_SCATTER) {
          float scatterDist = min_(-log_(xi_3) / m.mdensity, hDist);
          medS = scatterDist < hDist;
          if (medS) {
            transmittance *= exp_(-1.0f * scatterDist);
            hist = hist * (m.mcolor * transmittance);
            hP = hP + hV * scatterDist;
            f3 scatterDir = SampleHG(V, m.manis, sx, sy);
            scatter_pdf = PhaseHG(dot(V, scatterDir), m.manis);
            L = scatterDir;
          }
        }
        evf = DisneyEval(m, V, hN, L, evp);
        if (medS && scatter_pdf > 0.0f) {
          evp = scatter_pdf;
          evf = splat(scatter_pdf);
        }
        ro = hP;
        rd = L;
        phase = PH_CONT;
      } else {
        fin = Le0 + Lo;
        doFinish = true;
      }
    }

    // ------------------------------------------- progressive blend (RT:1552), next frame
    if (doFinish) {
      float n = (float)P.loop_num[frame];
      float a = 1.0f / n;
      float b = (float)(P.loop_num[frame] - 1) / n;
      acc = a * fin + b * acc;
      frame++;
      if (frame < P.n_frames) {
        phase = PH_START;
      } else {
        P.accum[accIdx] = make_float4(acc.x, acc.y, acc.z, 0.0f);
        phase = PH_IDLE;
      }
    }

    // -------------------------------------------------- pull pixels (wave-aggregated)
    const bool need = (phase == PH_IDLE) && !exhausted;
    const unsigned long long needMask = __ballot(need);
    if (needMask) {
      const int cnt = __popcll(needMask);
      const int leader = __ffsll((long long)needMask) - 1;
      unsigned int base = 0;
      if (lane == leader) base = atomicAdd(P.counter, (unsigned int)cnt);
      base = __shfl(base, leader);
      if (need) {
        unsigned int my = base + (unsigned int)__popcll(needMask & ((1ull << lane) - 1ull));
        if (my < P.n_work) {
          int lt = (int)(my / (unsigned)tpx);
          int r = (int)(my - (unsigned)lt * (unsigned)tpx);
          int gt = P.tile_ids[lt];
          int tx = gt % P.tiles_x, ty = gt / P.tiles_x;
          int blk = r >> 6, in = r & 63;
          int bxs = P.tile_w >> 3;
          int lx = (blk % bxs) * 8 + (in & 7);
          int ly = (blk / bxs) * 8 + (in >> 3);
          int px = tx * P.tile_w + lx, py = ty * P.tile_h + ly;
          if (px < P.W && py < P.H) {
            accIdx = lt * tpx + ly * P.tile_w + lx;
            float4 h = P.accum[accIdx];
            acc = mk3(h.x, h.y, h.z);
            u = ((float)px + 0.5f) / (float)P.W;  // TexCoords (vertex_shader.glsl, Screen.h:8-16)
            v = ((float)py + 0.5f) / (float)P.H;
            frame = 0;
            phase = PH_START;
          }
        } else {
          exhausted = true;
        }
      }
    }

    // ----------------------------------------------------------- camera ray (RT:1520-1528)
    if (phase == PH_START) {
      wseed = (uint32_t)(P.rand_origin[frame] * 6.95857f * (u * v));  // R5
      f3 lbc = mk3(P.lbc[0], P.lbc[1], P.lbc[2]);
      f3 right = mk3(P.right[0], P.right[1], P.right[2]);
      f3 up = mk3(P.up[0], P.up[1], P.up[2]);
      ro = camPos;
      rd = normalize(lbc + (u * 2.0f * P.half_w) * right + (v * 2.0f * P.half_h) * up);  // R6
      phase = PH_CAMERA;
      nsamples++;
    }

    const bool hasRay = phase == PH_CAMERA || phase == PH_SHADOW || phase == PH_CONT;
    if (!__any(hasRay)) {
      if (!__any(!exhausted)) break;
      continue;
    }
    if (hasRay) {
      trace<COUNT>(P, ro, rd, phase == PH_SHADOW, cull, sref, sdist, stride, trTri, trT, vis);
      nrays++;
    }
  }

  // one atomic per wave for the counters
  for (int off = 32; off > 0; off >>= 1) {
    nrays += __shfl_xor(nrays, off);
    nsamples += __shfl_xor(nsamples, off);
    if (COUNT) {
      vis.internal += __shfl_xor(vis.internal, off);
      vis.leaf += __shfl_xor(vis.leaf, off);
      vis.tri += __shfl_xor(vis.tri, off);
    }
  }
  if (lane == 0) {
    atomicAdd(&P.stats[0], nrays);
    atomicAdd(&P.stats[1], nsamples);
    if (COUNT) {
      atomicAdd(&P.stats[2], vis.internal);
      atomicAdd(&P.stats[3], vis.leaf);
      atomicAdd(&P.stats[4], vis.tri);
    }
  }
}

// Un-permute rank-major gathered tile buffers into a W x H x 3 fp32 frame.
// tile_src[global tile] = (owning rank, its local index there).
__global__ void rt_assemble_kernel(const float4* __restrict__ gathered, float* __restrict__ frame, int W, int H,
                                   int tile_w, int tile_h, int tiles_x, const int2* __restrict__ tile_src,
                                   int max_local_tiles) {
  int px = blockIdx.x * blockDim.x + threadIdx.x;
  int py = blockIdx.y;
  if (px >= W || py >= H) return;
  int tx = px / tile_w, ty = py / tile_h;
  int gt = ty * tiles_x + tx;
  const int2 src = tile_src[gt];
  int rank = src.x, lt = src.y;
  int lx = px - tx * tile_w, ly = py - ty * tile_h;
  size_t idx = ((size_t)rank * max_local_tiles + lt) * (size_t)(tile_w * tile_h) + (size_t)ly * tile_w + lx;
  float4 c = gathered[idx];
  size_t o = 3 * ((size_t)py * W + px);
  frame[o] = c.x;
  frame[o + 1] = c.y;
  frame[o + 2] = c.z;
}

// rt_update_materials: the material id lives in .w of each triangle's first normal texel
// (and of the shade's hit record, KParams::hrec)
__global__ __launch_bounds__(256) void rt_set_material_kernel(float4* __restrict__ trin, float4* __restrict__ hrec,
                                                             int first, int count, int id) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count) {
    trin[3 * (size_t)(first + i)].w = __int_as_float(id);
    hrec[8 * (size_t)(first + i) + 3].w = __int_as_float(id);
  }
}

// ------------------------------------------------------------ display (rt_tonemap)
// fragment_shader_tone_mapping.glsl:66-93 (simpleACES + pow 1/2.2) or the screen blit,
// GL unorm8 conversion, SaveFrame's vertical flip (out row 0 = top).  Reads either this
// rank's tile accumulation (world == 1) or an assembled H x W x 3 frame (row 0 = bottom).
RTD f3 simple_aces(f3 c) {  // TM:66-75
  const float a = 2.51f, b = 0.03f, y = 2.43f, d = 0.59f, e = 0.14f;
  const f3 num = c * (a * c + splat(b));
  const f3 den = c * (y * c + splat(d)) + splat(e);
  const f3 r = num / den;
  return mk3(clamp_(r.x, 0.0f, 1.0f), clamp_(r.y, 0.0f, 1.0f), clamp_(r.z, 0.0f, 1.0f));
}
RTD unsigned char unorm8(float f) { return (unsigned char)(int)(clamp_(f, 0.0f, 1.0f) * 255.0f + 0.5f); }

// NEE light samples per hdrCache texel (SampleHdrLight): the direction SampleHdr returns for the
// texel, and hdrColor / hdrPdf of that direction (hdrColorPdf) — the same device functions the
// shade would call, so the same bits.  Depends on envAngle: rebuilt when a call's angle changes.
__global__ __launch_bounds__(256) void rt_light_table_kernel(const Env E, float4* __restrict__ out) {
  const unsigned int n = (unsigned int)E.w * (unsigned int)E.h;
  for (unsigned int k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
    const f3 L = SampleHdrTexel(E.cache[k]);
    f3 color;
    float pdf;
    hdrColorPdf(E, L, color, pdf);
    out[2u * k] = make_float4(L.x, L.y, L.z, pdf);
    out[2u * k + 1u] = make_float4(color.x, color.y, color.z, 0.0f);
  }
}

__global__ __launch_bounds__(256) void rt_display_kernel(const float4* __restrict__ tiles, const float* __restrict__ frame,
                                                         unsigned char* __restrict__ out, int W, int H, int tile_w,
                                                         int tile_h, int tiles_x, int flags) {
  const int px = blockIdx.x * blockDim.x + threadIdx.x, py = blockIdx.y;
  if (px >= W || py >= H) return;
  f3 c;
  if (tiles) {
    const int tx = px / tile_w, ty = py / tile_h;
    const size_t idx = (size_t)(ty * tiles_x + tx) * (size_t)(tile_w * tile_h) +
                       (size_t)(py - ty * tile_h) * tile_w + (px - tx * tile_w);
    const float4 v = tiles[idx];
    c = mk3(v.x, v.y, v.z);
  } else {
    const float* p = frame + 3 * ((size_t)py * W + px);
    c = mk3(p[0], p[1], p[2]);
  }
  if (flags & 1) {
    c = simple_aces(c);
    if (flags & 2) {
      const float g = 1.0f / 2.2f;
      c = mk3(pow_(c.x, g), pow_(c.y, g), pow_(c.z, g));
    }
  }
  unsigned char* o = out + 3 * ((size_t)(H - 1 - py) * W + px);
  o[0] = unorm8(c.x);
  o[1] = unorm8(c.y);
  o[2] = unorm8(c.z);
}

}  // namespace rtd
