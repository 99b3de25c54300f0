// rt_wavefront.h — wavefront formulation of the path tracer for gfx950.
//
// The reference runs one fragment per pixel that loops over bounces (RT:1369-1516).  On a
// 64-wide wavefront that megakernel form mixes traversal with long, divergent shading code and
// pins ~170 VGPRs for the whole path.  Here a frame is a sequence of small kernels over
// device-resident path state (one slot per pixel of this rank):
//
//   wf_camera  camera ray direction and u*v per pixel (RT:1520-1527)  -> per-pixel table
//   wf_trace   closest-hit / any-hit BVH traversal of every queued   -> (triangle, t) per ray
//              ray, persistent grid with per-lane dynamic ray fetch
//   wf_shade   per active path: apply the NEE result (RT:1389-1405),  -> next rays, next list
//              the medium-emissive term (RT:1437-1439), the continuation result (RT:1483-1510),
//              then the next bounce's light sample, DisneySample, media and DisneyEval
//              (RT:1376-1474); finished paths blend into the accumulation (RT:1552)
//
// wf_trace + wf_shade repeat maxBounce+1 times; passes with no work exit at once.  All frames
// of one launch are in flight together (path slot = pixel * n_frames + frame): a pixel's frames
// are independent until the progressive blend, so wf_blend applies RT:1552 afterwards in frame
// order, exactly as sequential frames would.  This amortises the serial tail of the deepest
// rays of each pass over several frames.  Shadow and continuation rays of all paths share one
// traversal launch.  Every value that
// reaches the image is computed with the same fp32 operations, in the same order, as the
// oracle (the pending NEE term is added to Lo before the medium term and before the
// continuation term, as in the shader), so results stay bit-identical.
#pragma once
#include "rt_kernels.h"

namespace rtd {

// RT_CHECK (development build: make variant HIPEXTRA=-DRT_CHECK): bounds checks that report the
// first bad index of a launch with printf and replace it with a harmless one instead of faulting

// per-path flags (< 256: packed with the bounce in s5.y)
enum : uint32_t {
  PF_SHADOW = 1u,      // a shadow ray was traced for the current bounce (c_nee pending)
  PF_CMED = 2u,        // medium-emissive term pending (RT:1438)
  PF_CONT = 4u,        // a continuation ray is queued (else the path ends after the shadow ray)
  PF_MEDIUM = 8u,      // mediumSampled (RT:1444)
  PF_CAMERA = 16u,     // the queued continuation ray is the camera ray
  PF_ZLO = 32u         // Lo and Le0 are +0 (all bits): s1 not stored, s3 only with a shadow ray
};

struct WFState {
  float4* __restrict__ s0;   // hist.xyz, evp
  float4* __restrict__ s1;   // Lo.xyz, Le0.x
  float4* __restrict__ s2;   // evf.xyz, Le0.y
  float4* __restrict__ s3;   // cnee.xyz, Le0.z
  float4* __restrict__ s4;   // cmed.xyz, -
  uint2* __restrict__ s5;    // wseed, bounce << 8 | flags (the frame is slot % frames: pixel-major)
  // rays in 24 B: {o.xyz, d.x} + {d.y, d.z} (continuation ra/rb, shadow sa/sb); 32 B as two
  // float4 cost the memory-bound shade 16 B of writes and 8 B of reads per path-bounce
  float4* __restrict__ ra;
  float2* __restrict__ rb;
  float4* __restrict__ sa;
  float2* __restrict__ sb;
  // per path: [2*p + 0] the continuation's closest triangle, [2*p + 1] the shadow ray's (-1: none).
  // The hit distance is not stored: the shade recomputes t from that triangle and the ray with the
  // traversal's own operations (RT:265), the same bits (4 B per ray written instead of 8)
  int* __restrict__ res;
  float4* __restrict__ fin;  // per path: final radiance curColor (RT:1549) awaiting the blend
  const unsigned int* __restrict__ pix_xy;   // per work item: px | py << 16
  const unsigned int* __restrict__ pix_acc;  // per work item: accumulation index
  float4* __restrict__ cam;                   // per work item: camera direction, u * v (wf_camera)
  // per work item: the camera hit point of its pixel (pass 0's shade, frame 0 of each pixel).  All
  // of a pixel's frames share it (R6: the camera ray is the same in every frame), so the rays that
  // pass 0 queues are stored as 16 B: {d.xyz, s} in ra / sa, origin = org + cam.xyz * s (s = the
  // medium scattering distance of a continuation, else 0) instead of {o.xyz, d.x} + {d.y, d.z}
  float4* __restrict__ org;
  int* queue[2];                // ray queue entries: path << 1 | is_shadow
  int* queue_s[2];              // split queues (WFParams::split): the shadow rays, queue[k] + slots
  int* active[2];               // active path ids
  unsigned int* __restrict__ cnt;  // queue counts, active counts, trace fetch, segment claims (cq, ca, ... below)
};

constexpr int kFlagNoRayHist = 1 << 30;  // (internal, development builds) KParams::flags: no per-ray histogram

// WFState::cnt words: the ray-queue counts of the two pass parities (cq), the active-list counts
// (ca), the trace's / finisher's fetch counter and the claim counters of the 8 queue segments
// (xcnt), one 128-B line each: a device-scope atomic occupies its line ~11 ns (88
// per us per line, whatever the word, and lines scale: tools/atomic_bench.hip,
// profiles/r05_atomic_throughput.log).  (The pass counters on lines of their own measured
// neutral, round 5.)
__host__ __device__ constexpr unsigned int cq(unsigned int i) { return i; }
__host__ __device__ constexpr unsigned int ca(unsigned int i) { return 2u + i; }
constexpr unsigned int kCntFetch = 4u;
__host__ __device__ constexpr unsigned int xcnt(unsigned int s) { return 160u + 32u * s; }
// split queues (WFParams::split): the shadow-ray queue counts of the two parities, and the claim
// counters of its 8 segments (the continuation queue keeps cq / xcnt)
__host__ __device__ constexpr unsigned int cqs(unsigned int i) { return 6u + i; }
__host__ __device__ constexpr unsigned int xcnts(unsigned int s) { return 416u + 32u * s; }
constexpr unsigned int kCntWords = 416u + 32u * 8u;

// Per-wave statistics flushes of wf_shade / wf_finish (rays, samples, finisher steps) go to one of
// kStatShards 128-B lines after the 128 counters (words 0, 1, 2 of shard s = rays, samples, finish
// steps), summed by the host, instead of all waves of a launch's end queueing at one line: C3
// 1080p one-frame calls -6.1% (2.488 -> 2.335 ms synchronised), bulk +0.17% (round 5,
// profiles/r05_ab_stats_shards_C3.log)
constexpr unsigned int kStatShards = 64u, kStatWords = 128u + 16u * kStatShards;
__host__ __device__ constexpr unsigned int stats_shard(unsigned int wave) { return 128u + 16u * (wave % kStatShards); }

// a ray queued by pass 0 in the 16-B form (see WFState::org): origin and direction
RTD void p1_ray(const WFState& S, unsigned int n_frames, unsigned int path, const float4 a, float& ox, float& oy,
                float& oz) {
  const unsigned int w = path / n_frames;
  const float4 o = S.org[w];
  ox = o.x; oy = o.y; oz = o.z;
  if (a.w != 0.0f) {  // a scattered continuation: hP + hV * scatterDist, as pass 0's shade computed it
    const float4 c = S.cam[w];
    ox = o.x + c.x * a.w; oy = o.y + c.y * a.w; oz = o.z + c.z * a.w;
  }
}
// path-state and ray stores of the shade step: non-temporal with RT_SHADE_NT (rows written once
// per pass and read by the next pass's kernels, after they have left the caches)
#ifndef RT_SHADE_NT  // C3 bulk +1.13%, one-frame calls +0.3% (noise) (profiles/r04_ab_nt_shade_stores_C3.log)
#define RT_SHADE_NT 1
#endif
typedef float nt_f4 __attribute__((ext_vector_type(4)));
typedef float nt_f2 __attribute__((ext_vector_type(2)));
typedef unsigned int nt_u2 __attribute__((ext_vector_type(2)));
RTD void st_row(float4* p, float4 v) {
  if (RT_SHADE_NT) __builtin_nontemporal_store(nt_f4{v.x, v.y, v.z, v.w}, reinterpret_cast<nt_f4*>(p));
  else *p = v;
}
RTD void st_row(float2* p, float2 v) {
  if (RT_SHADE_NT) __builtin_nontemporal_store(nt_f2{v.x, v.y}, reinterpret_cast<nt_f2*>(p));
  else *p = v;
}
RTD void st_row(uint2* p, uint2 v) {
  if (RT_SHADE_NT) __builtin_nontemporal_store(nt_u2{v.x, v.y}, reinterpret_cast<nt_u2*>(p));
  else *p = v;
}
RTD void put_ray(float4* a, float2* b, unsigned int p, float ox, float oy, float oz, float dx, float dy, float dz) {
  st_row(a + p, make_float4(ox, oy, oz, dx));
  st_row(b + p, make_float2(dy, dz));
}

struct WFParams {
  KParams K;  // scene, env, camera, frame geometry; K.n_work = valid pixels of this rank
  WFState S;
  int n_frames;  // frames in flight: slots = n_frames * K.n_work
  int pass;      // bounce pass: queue/active set pass&1 in, (pass+1)&1 out
  // implicit camera pass: when nonzero, this pass's ray queue and active list are the camera
  // paths of slots [0, cam_n) in slot order (entry i = slot i), generated where they are used
  // (wf_trace refill, wf_shade) instead of being written by a generation kernel and read back
  unsigned int cam_n;
  int p1_compact;  // pass 0 queues 16-B rays from the per-pixel origin (off when the finisher starts at pass 1)
  // one frame per path-state set and nothing in flight before it (unpipelined calls of one frame
  // per group): a finishing path blends into the accumulation itself (wf_blend's operations,
  // RT:1552) instead of writing fin for a wf_blend launch after the last pass
  int fuse_blend;
  // bulk groups: the shade queues shadow rays (queue_s, cqs) and continuations (queue, cq) apart,
  // and each secondary pass traces them in two launches, wf_trace<..., KIND = 2> and <..., 1>.
  // split: this pass's rays are in split queues; split_out: the shade queues the next pass's apart
  int split, split_out;
};

// Map a work index of this rank to (pixel, accumulation index); false outside the frame.
RTD bool work_pixel(const KParams& P, unsigned int w, int& px, int& py, int& accIdx) {
  const int tpx = P.tile_w * P.tile_h;
  int lt = (int)(w / (unsigned)tpx);
  int r = (int)(w - (unsigned)lt * (unsigned)tpx);
  int gt = P.tile_ids[lt];
  int tx = gt % P.tiles_x, ty = gt / P.tiles_x;
  int blk = r >> 6, in = r & 63;
  int bxs = P.tile_w >> 3;
  int lx = (blk % bxs) * 8 + (in & 7);
  int ly = (blk / bxs) * 8 + (in >> 3);
  px = tx * P.tile_w + lx;
  py = ty * P.tile_h + ly;
  accIdx = lt * tpx + ly * P.tile_w + lx;
  return px < P.W && py < P.H;
}

// wave-aggregated append of `want` lanes to a counter; returns this lane's slot
RTD unsigned int wave_append(unsigned int* counter, bool want) {
  const unsigned long long m = __ballot(want);
  unsigned int base = 0;
  if (m) {
    const int lane = (int)(threadIdx.x & 63);
    const int leader = __ffsll((long long)m) - 1;
    if (lane == leader) base = atomicAdd(counter, (unsigned int)__popcll(m));
    base = __shfl(base, leader);
    base += (unsigned int)__popcll(m & ((1ull << lane) - 1ull));
  }
  return base;
}

// Wave-aggregated append into a block-local LDS list: every lane of the wave calls it
// (wave-uniform control flow) with n = 0, 1 or 2 entries; one LDS atomic per wave.
RTD unsigned int wave_lds_append(unsigned int* lcount, unsigned int n) {
  const int lane = (int)(threadIdx.x & 63);
  const unsigned long long b1 = __ballot(n >= 1u), b2 = __ballot(n >= 2u);
  const unsigned long long below = (1ull << lane) - 1ull;
  const unsigned int mine = (unsigned int)(__popcll(b1 & below) + __popcll(b2 & below));
  const unsigned int wtot = (unsigned int)(__popcll(b1) + __popcll(b2));
  unsigned int base = 0;
  if (lane == 0 && wtot) base = atomicAdd(lcount, wtot);
  return (unsigned int)__shfl((int)base, 0) + mine;
}

// Per work item of this rank: the camera ray direction and u*v of its pixel (RT:1520-1527),
// written once per render call; every frame's camera ray of that pixel reads it.  Block 0 also
// zeroes the batch's groups' pass counters (16 words each: no memset ahead of each group's passes).
struct GroupCounters {
  unsigned int* cnt[4];
  int n;
};
__global__ __launch_bounds__(256) void wf_camera(const WFParams W, const GroupCounters Z) {
  const KParams& P = W.K;
  const WFState& S = W.S;
  if (blockIdx.x == 0)
    for (unsigned int i = threadIdx.x; i < kCntWords * (unsigned)Z.n; i += blockDim.x) Z.cnt[i / kCntWords][i % kCntWords] = 0u;
  const f3 lbc = mk3(P.lbc[0], P.lbc[1], P.lbc[2]);
  const f3 right = mk3(P.right[0], P.right[1], P.right[2]);
  const f3 up = mk3(P.up[0], P.up[1], P.up[2]);
  for (unsigned int w = blockIdx.x * blockDim.x + threadIdx.x; w < P.n_work; w += gridDim.x * blockDim.x) {
    const unsigned int xy = S.pix_xy[w];
    const int px = (int)(xy & 0xffffu), py = (int)(xy >> 16);
    const float u = ((float)px + 0.5f) / (float)P.W;  // TexCoords (vertex_shader.glsl)
    const float v = ((float)py + 0.5f) / (float)P.H;
    const f3 d = normalize(lbc + (u * 2.0f * P.half_w) * right + (v * 2.0f * P.half_h) * up);  // R6
    S.cam[w] = make_float4(d.x, d.y, d.z, u * v);
  }
}

// Per frame of a render call: sobolVec2(loopNum + 1, bounce) of RT:616-620 for bounces 0..3
// (Sobol dims 0..7), so wf_shade reads one float2 instead of running two bit loops per bounce.
// Also the blend weights of each frame, {1 / n, (n - 1) / n} with n = loopNum (RT:1552), the same
// operations wf_blend would run per pixel.
// A call of at most RT_INLINE_FRAMES frames passes its (loopNum, randOrigin) pairs as kernel
// arguments and this kernel writes them into the device frame table (no host-to-device copies in
// a one-frame call's critical path); larger calls upload the table first (F.n_inline = 0).
#ifndef RT_INLINE_FRAMES
#define RT_INLINE_FRAMES 8
#endif
struct InlineFrames {
  int n_inline;
  int loop[RT_INLINE_FRAMES];
  float ro[RT_INLINE_FRAMES];
};
__global__ __launch_bounds__(256) void wf_sobol(int* __restrict__ loop_num, float* __restrict__ rand_origin,
                                                float2* __restrict__ out, float2* __restrict__ blend_w, int n_frames,
                                                const InlineFrames F) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool inl = F.n_inline > 0;
  if (i < n_frames) {
    const int loopNum = inl ? F.loop[i] : loop_num[i];
    if (inl) {
      loop_num[i] = loopNum;
      rand_origin[i] = F.ro[i];
    }
    const float n = (float)loopNum;
    blend_w[i] = make_float2(1.0f / n, (float)(loopNum - 1) / n);
  }
  if (i >= n_frames * 4) return;
  int g = (inl ? F.loop[i >> 2] : loop_num[i >> 2]) + 1;
  g = g ^ (g >> 1);  // grayCode (RT:598-600)
  const int b = i & 3;
  out[i] = make_float2(sobol_gray(2 * b, g), sobol_gray(2 * b + 1, g));
}
RTD void sobol_pair(const KParams& P, uint32_t frame, uint32_t bounce, float& sx, float& sy) {
  sx = sy = 0.0f;  // bounce >= 4 reads dims >= 8: outside the table (R8)
  if (bounce < 4u) {
    const float2 s = P.sobol[frame * 4u + bounce];
    sx = s.x;
    sy = s.y;
  }
}

// Camera ray of path slot `slot`: direction, seed (R5) and frame of the slot.  Path slots are
// pixel-major (slot = work item * n_frames + frame): the camera pass hands a wave one pixel's
// frames, whose camera rays are the same ray (R6: no jitter), so its lanes traverse in lockstep,
// and the next passes start from the same hit point.
RTD f3 camera_ray(const KParams& P, const WFState& S, unsigned int slot, uint32_t& wseed, uint32_t& frame) {
  const unsigned int nf = (unsigned int)P.n_frames;
  const unsigned int w = slot / nf;
  const unsigned int f = slot - w * nf;
  const float4 c = S.cam[w];
  wseed = (uint32_t)(P.rand_origin[f] * 6.95857f * c.w);  // R5: rand_origin * 6.95857 * (u * v)
  frame = f;
  return xyz(c);
}

// progressive blend of the frames in flight, in frame order (RT:1552).  Pixel-major slots put
// a pixel's frames side by side, so the block stages 8 frames of its 256 pixels at a time in LDS
// with whole-cache-line loads (8 lanes per pixel) and each thread then blends its own pixel.
// The next stage's loads are issued into registers before the current stage is blended, so the
// HBM latency overlaps the blend (C3 bulk +0.88%, round 5, profiles/r05_ab_bulk_blend_prefetch_C3.log;
// the stage's blend weights come through LDS: vector-memory waits are in order, so a weight load
// issued after the prefetch would wait for it too).
constexpr int BL_FR = 8, BL_PITCH = BL_FR + 1;  // frames per stage; padded row (bank spread)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void wf_blend(const WFParams W) {
  __shared__ float4 tile[256 * BL_PITCH];
  const KParams& P = W.K;
  const WFState& S = W.S;
  const unsigned int nf = (unsigned int)W.n_frames;
  for (unsigned int base = blockIdx.x * 256u; base < P.n_work; base += gridDim.x * 256u) {
    const unsigned int w = base + threadIdx.x;
    const bool valid = w < P.n_work;
    const unsigned int ai = valid ? S.pix_acc[w] : 0u;
    f3 acc = splat(0.0f);
    if (valid) {
      const float4 h = P.accum[ai];
      acc = mk3(h.x, h.y, h.z);
    }
    {
      static_assert(BL_FR == 8, "eight named registers");
      // (unconditional loads from a clamped index: a branch around each load would make the
      // compiler wait for all of them before the blend below; named registers, not an array:
      // a loop-carried private array stayed in scratch)
      float4 r0, r1, r2, r3, r4, r5, r6, r7;
      __shared__ float2 wst[BL_FR];
      auto ld1 = [&](unsigned int f0, int j) {
        const unsigned int nfc = min((unsigned int)BL_FR, nf - f0);
        const unsigned int i = threadIdx.x + 256u * (unsigned)j, p = i / BL_FR, k = i % BL_FR;
        const bool ok = base + p < P.n_work && k < nfc;
        return S.fin[ok ? (size_t)(base + p) * nf + f0 + k : 0];
      };
      auto st1 = [&](int j, float4 v) {
        const unsigned int i = threadIdx.x + 256u * (unsigned)j, p = i / BL_FR, k = i % BL_FR;
        tile[p * BL_PITCH + k] = v;
      };
#define RT_BLEND_FETCH(F0)                                                                          \
  {                                                                                                 \
    r0 = ld1(F0, 0); r1 = ld1(F0, 1); r2 = ld1(F0, 2); r3 = ld1(F0, 3);                             \
    r4 = ld1(F0, 4); r5 = ld1(F0, 5); r6 = ld1(F0, 6); r7 = ld1(F0, 7);                             \
  }
      RT_BLEND_FETCH(0u)
      for (unsigned int f0 = 0; f0 < nf; f0 += BL_FR) {
        const unsigned int nfc = min((unsigned int)BL_FR, nf - f0);
        __syncthreads();
        st1(0, r0); st1(1, r1); st1(2, r2); st1(3, r3); st1(4, r4); st1(5, r5); st1(6, r6); st1(7, r7);
        // (read from LDS after the barrier: a vector-memory load of them after the prefetch below
        // would wait for the prefetch too, vmcnt being in order)
        if (threadIdx.x < (unsigned)BL_FR) wst[threadIdx.x] = P.blend_w[f0 + (threadIdx.x < nfc ? threadIdx.x : 0u)];
        __syncthreads();
        float2 bw[BL_FR];  // the stage's blend weights {1 / n, (n - 1) / n}, staged in LDS with the tile
#pragma unroll
        for (int k = 0; k < BL_FR; k++) bw[k] = wst[k];
        if (f0 + BL_FR < nf) RT_BLEND_FETCH(f0 + BL_FR)
#undef RT_BLEND_FETCH
        if (valid)
#pragma unroll
          for (int k = 0; k < BL_FR; k++) {
            if ((unsigned)k < nfc) {
              const float4 c = tile[threadIdx.x * BL_PITCH + k];
              acc = bw[k].x * xyz(c) + bw[k].y * acc;
            }
          }
      }
    }
    if (valid) P.accum[ai] = make_float4(acc.x, acc.y, acc.z, 0.0f);
  }
}

// ----------------------------------------------------------------------------- trace
// Persistent traversal: every lane pulls queued rays (one atomic per 64 rays per wave) and
// runs the reference's near-first DFS (RT:338-390) with culling of subtrees that start beyond
// the current closest hit (culling only drops subtrees whose entry distance exceeds the best
// hit so far, so the closest hit is the reference's).  The wave schedule is the dual cursor:
// every lane keeps a traversal cursor and a triangle cursor and each iteration advances both (one
// triangle of the current leaf + one node step); a lane waits only when it reaches a second leaf
// before finishing the first, and idle lanes refill from the queue.  (Measured and removed: the
// if-if schedule, while-while and Aila & Laine's speculative while-while)

struct TraceLane {
  // ray as scalars (f3 members made SROA keep the lane in scratch memory)
  float ox, oy, oz, dx, dy, dz, ix, iy, iz;
  RTD f3 o() const { return mk3(ox, oy, oz); }
  RTD f3 d() const { return mk3(dx, dy, dz); }
  RTD f3 inv() const { return mk3(ix, iy, iz); }
  float best, bestt;
  // cull_limit of the current best, kept per ray (1 VGPR) and updated when best changes instead of
  // recomputed at every use: C3 bulk +0.58% (round 5, profiles/r05_ab_bulk_cached_limit_C3.log;
  // round 2's attempt spilled)
  float lim;
  RTD float limit(float) const { return lim; }
  RTD void set_best(float d, float eps) {
    best = d;
    lim = cull_limit(d, eps, ix, iy, iz);
  }
  int besttri, sp, cur, tri_i, tri_end;
  int offNx, offNy, offNz;  // byte offset, inside a QNode, of the near-plane float4 of each axis
  bool haveCur, anyhit, finite;
};

typedef float v2f __attribute__((ext_vector_type(2)));

// Traversal stack of one lane: entries [0, KL) in LDS at lds[j * TL_LANES] ([entry][lane], the
// block is always 256 lanes, so addresses are shifts), deeper ones in the global overflow
// column (explicitly global, so the accesses never become FLAT and never wait on LDS counters).
typedef __attribute__((address_space(1))) unsigned long long gu64;  // {ref, key} packed
RTD unsigned long long pack_ent(int2 e) { return (unsigned long long)(uint32_t)e.x | ((unsigned long long)(uint32_t)e.y << 32); }
RTD int2 unpack_ent(unsigned long long v) { return make_int2((int)(uint32_t)v, (int)(uint32_t)(v >> 32)); }
constexpr int TL_LANES = 256;
RTD uint32_t lds_addr(const void* p) { return (uint32_t)(size_t)(const __attribute__((address_space(3))) void*)p; }
struct TraceStack {
  int2* lds;      // this lane's column: entry j at lds[j * TL_LANES]
  int2* lds0;     // the block's stack (lane 0's column)
  gu64* ovf;      // the block's overflow columns: entry j >= KL of block lane l at ovf[(j - KL) * ovs + l]
  unsigned ovs;
  int KL;
#ifdef RT_CHECK
  int cap;  // KParams::stack_cap: the overflow columns hold entries KL .. cap - 1
#endif
  RTD uint32_t lane() const {
    uint32_t l = (lds_addr(lds) - lds_addr(lds0)) >> 3;
    asm volatile("" : "+v"(l));  // recomputed where used: a hoisted 64-bit address would live in scratch
    return l;
  }
  // the overflow slot of entry j (the lane from the LDS column: no 64-bit per-lane pointer lives
  // across the traversal loop)
  RTD gu64* ovf_at(int j) const {
#ifdef RT_CHECK
    if (j < KL || j >= cap) printf("[rt check] overflow stack index %d (KL %d, cap %d)\n", j, KL, cap);
#endif
    return ovf + (size_t)(j - KL) * ovs + lane();
  }
};

// byte-offset loads from a uniform base: the compiler emits the saddr form (32-bit lane offset)
template <class T>
RTD T ld(const void* base, uint32_t byte_off) {
  return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + byte_off);
}

// Exact-tie rule of the reference traversal (only the 4-wide schedule needs it: it visits
// leaves in a different order).  The reference keeps the FIRST of equally distant hits in its
// near-first DFS order (RT:328 / RT:356 use strict <).  Two triangles in one leaf: lower index
// first.  Otherwise descend the binary tree to the node whose children separate the two
// leaves (GNode.ref.z = DFS rank of the first right-subtree leaf): the reference enters the
// left child first iff d1 < d2 (RT:373-382; both children were reached, so both d > 0).
RTD bool tie_wins(const KParams& P, const TraceLane& L, int a, int b) {
  const int ra = __float_as_int(P.trin[3 * a + 1].w), rb = __float_as_int(P.trin[3 * b + 1].w);
  if (ra == rb) return a < b;
  int node = P.root;
  for (int guard = 0; guard < 64 && !ref_is_leaf(node); guard++) {
    const GNode g = ld<GNode>(P.nodes, (uint32_t)node * 64u);
    const bool aL = ra < g.ref.z, bL = rb < g.ref.z;
    if (aL == bL) {
      node = aL ? g.ref.x : g.ref.y;
      continue;
    }
    float e1, e2;
    const float d1 = slab(L.o(), L.inv(), mk3(g.b0.x, g.b0.y, g.b0.z), mk3(g.b0.w, g.b1.x, g.b1.y), e1);
    const float d2 = slab(L.o(), L.inv(), mk3(g.b1.z, g.b1.w, g.b2.x), mk3(g.b2.y, g.b2.z, g.b2.w), e2);
    return aL == (d1 < d2);
  }
  return a < b;
}

// The reference's three edge functions (RT:273-281) on the computed hit point: only for the
// points the barycentric filter below cannot decide (p2, p3 from the shading record P.tri).
RTD bool tl_edges_exact(const KParams& P, int i, const f3 p1, const f3 ng, const f3 Pp) {
  const uint32_t off = (uint32_t)i * 48u;
  const f3 p2 = xyz(ld<float4>(P.tri, off + 16u)), p3 = xyz(ld<float4>(P.tri, off + 32u));
  const float e1 = dot(cross(p2 - p1, Pp - p1), ng);
  const float e2 = dot(cross(p3 - p2, Pp - p2), ng);
  const float e3 = dot(cross(p1 - p3, Pp - p3), ng);
  return (e1 > 0 && e2 > 0 && e3 > 0) || (e1 < 0 && e2 < 0 && e3 < 0);
}

// one triangle (RT:241-299, R1); true when it becomes the closest hit.  {A, B, Cc} = the traversal
// record {p1, Ng.x} {R2, Ng.y} {R3, Ng.z} (csrc/common/tri_filter.h): the plane test and t are the
// reference's operations; "inside" is decided by the barycentric rows b2 = R2.(P - p1),
// b3 = R3.(P - p1), b1 = 1 - b2 - b3 whenever min(b) lies outside the error margin
// m = k1 * max|P - p1| * (max|R2| + max|R3|) + k0 that bounds both b's error and the fp32 error of
// the reference's edge functions (tri_filter.h derives it), else by those edge functions.
// the hit test alone (no tie rule, L unchanged): true when triangle i is hit at dist <= L.best
// (WIDE) / < L.best; dist = t - 0.00001 and t returned
template <bool WIDE>
RTD bool tl_tri_hit(const KParams& P, const TraceLane& L, int i, const float4 A, const float4 B, const float4 Cc,
                    float& dist_out, float& t_out) {
  const f3 p1 = xyz(A);
  const f3 ng = mk3(A.w, B.w, Cc.w);
  const float dn = dot(ng, L.d());
  const float num = dot(ng, p1) - dot(L.o(), ng);
  const float t = num / dot(L.d(), ng);                                // RT:265
  const float dist = t - 0.00001f;
  bool ok = !(fabs_(dn) < 0.00001f) & (t >= 0.0005f) & (WIDE ? dist <= L.best : dist < L.best);  // RT:262, 268, 328/356
  const f3 Pp = L.o() + L.d() * t;
  const float qx = Pp.x - p1.x, qy = Pp.y - p1.y, qz = Pp.z - p1.z;
  const float b2 = __builtin_fmaf(B.x, qx, __builtin_fmaf(B.y, qy, B.z * qz));
  const float b3 = __builtin_fmaf(Cc.x, qx, __builtin_fmaf(Cc.y, qy, Cc.z * qz));
  const float b1 = (1.0f - b2) - b3;
  const float mn = fminf(b1, fminf(b2, b3));
  const float dq = fmaxf(fabsf(qx), fmaxf(fabsf(qy), fabsf(qz)));
  const float lr = fmaxf(fabsf(B.x), fmaxf(fabsf(B.y), fabsf(B.z))) + fmaxf(fabsf(Cc.x), fmaxf(fabsf(Cc.y), fabsf(Cc.z)));
  const float m = (dq * lr) * P.tri_k1 + P.tri_k0;
  bool inside = mn > 0.0f;
  if (ok & !((fabsf(mn) > m) & (m < 0.25f))) inside = tl_edges_exact(P, i, p1, ng, Pp);
  dist_out = dist;
  t_out = t;
  return ok & inside;
}
// AH (the any-hit kernel of split queues, wf_trace<..., KIND = 2>): best is +inf until the hit that
// ends the ray, so `dist <= best` is the NaN test `t >= 0.0005` already makes and there is no tie;
// the accepted triangle ends the ray (no culling limit to update)
template <bool WIDE, bool AH = false>
RTD bool tl_triangle_calc(const KParams& P, TraceLane& L, int i, const float4 A, const float4 B, const float4 Cc) {
  // straight-line form: every condition of RT:262-281 folded into one predicate (a 64-lane wave
  // runs the whole test for some lane anyway; early returns, and round 2's rcp-based pre-reject
  // ahead of the division, only cost exec-mask juggling: +1.3% C3, profiles/r03_ab_bulk_tri_flat_C3.log)
  const f3 p1 = xyz(A);
  const f3 ng = mk3(A.w, B.w, Cc.w);
  const float dn = dot(ng, L.d());
  const float num = dot(ng, p1) - dot(L.o(), ng);
  const float t = num / dot(L.d(), ng);                                // RT:265
  const float dist = t - 0.00001f;
  bool ok = !(fabs_(dn) < 0.00001f) & (t >= 0.0005f) & (AH || (WIDE ? dist <= L.best : dist < L.best));  // RT:262, 268, 328/356
  const f3 Pp = L.o() + L.d() * t;
  const float qx = Pp.x - p1.x, qy = Pp.y - p1.y, qz = Pp.z - p1.z;
  const float b2 = __builtin_fmaf(B.x, qx, __builtin_fmaf(B.y, qy, B.z * qz));
  const float b3 = __builtin_fmaf(Cc.x, qx, __builtin_fmaf(Cc.y, qy, Cc.z * qz));
  const float b1 = (1.0f - b2) - b3;
  const float mn = fminf(b1, fminf(b2, b3));
  const float dq = fmaxf(fabsf(qx), fmaxf(fabsf(qy), fabsf(qz)));
  const float lr = fmaxf(fabsf(B.x), fmaxf(fabsf(B.y), fabsf(B.z))) + fmaxf(fabsf(Cc.x), fmaxf(fabsf(Cc.y), fabsf(Cc.z)));
  const float m = (dq * lr) * P.tri_k1 + P.tri_k0;
  bool inside = mn > 0.0f;
  if (ok & !((fabsf(mn) > m) & (m < 0.25f))) inside = tl_edges_exact(P, i, p1, ng, Pp);
  ok &= inside;
  if (AH) {
    if (ok) L.besttri = i;
    return ok;
  }
  if (WIDE && ok && dist == L.best) ok = L.besttri >= 0 && tie_wins(P, L, i, L.besttri);
  if (ok) {
    L.set_best(dist, P.cull_eps);
    L.besttri = i;
    L.bestt = t;
  }
  return ok;
}
template <bool WIDE, bool AH = false>
RTD bool tl_triangle(const KParams& P, TraceLane& L, int i) {
  const uint32_t off = (uint32_t)i * 48u;
  const float4 A = ld<float4>(P.trx, off), B = ld<float4>(P.trx, off + 16u), Cc = ld<float4>(P.trx, off + 32u);
  return tl_triangle_calc<WIDE, AH>(P, L, i, A, B, Cc);
}

RTD void tl_push(TraceLane& L, const TraceStack& S, int2 ent) {
  if (L.sp < S.KL) S.lds[L.sp * TL_LANES] = ent;
  else *S.ovf_at(L.sp) = pack_ent(ent);
  ++L.sp;
}

// pop the next surviving subtree (RT:348); false when the stack is exhausted
RTD bool tl_pop(const KParams& P, TraceLane& L, const TraceStack& S, bool cull) {
  const float lim = L.limit(P.cull_eps);
  while (L.sp > 0) {
    --L.sp;
    const int2 ent = L.sp < S.KL ? S.lds[L.sp * TL_LANES] : unpack_ent(*S.ovf_at(L.sp));
    if (cull && __int_as_float(ent.y) > lim) continue;
    L.cur = ent.x;
    return true;
  }
  return false;
}

// internal node L.cur (RT:361-385): both child boxes, near child first, far child stacked
RTD void tl_node(const KParams& P, TraceLane& L, const TraceStack& S, bool cull) {
  const uint32_t off = (uint32_t)L.cur * 64u;
  const float4 b0 = ld<float4>(P.nodes, off), b1 = ld<float4>(P.nodes, off + 16u), b2 = ld<float4>(P.nodes, off + 32u);
  const int2 ref = ld<int2>(P.nodes, off + 48u);
  float e1, e2;
  const float d1 = slab(L.o(), L.inv(), mk3(b0.x, b0.y, b0.z), mk3(b0.w, b1.x, b1.y), e1);
  const float d2 = slab(L.o(), L.inv(), mk3(b1.z, b1.w, b2.x), mk3(b2.y, b2.z, b2.w), e2);
  int nearRef = 0;
  float nearE = 0.0f;
  bool descend = false;
  if (d1 > 0 && d2 > 0) {  // RT:373-382
    const bool leftFirst = d1 < d2;
    nearRef = leftFirst ? ref.x : ref.y;
    nearE = leftFirst ? e1 : e2;
    tl_push(L, S, make_int2(leftFirst ? ref.y : ref.x, __float_as_int(leftFirst ? e2 : e1)));
    descend = true;
  } else if (d1 > 0) {
    nearRef = ref.x; nearE = e1; descend = true;
  } else if (d2 > 0) {
    nearRef = ref.y; nearE = e2; descend = true;
  }
  if (descend && cull && nearE > L.limit(P.cull_eps)) descend = false;
  L.cur = nearRef;
  L.haveCur = descend || tl_pop(P, L, S, cull);
}

// 4-wide node L.cur: the four (grand)child boxes of the binary subtree it replaces, each with
// the reference's slab test; survivors sorted by entry distance, nearest entered, rest stacked.
// Split in parts: the box tests (tl_qnode_keys, planes given), the sort + push (tl_qnode_push),
// so the finisher can fetch the node before its triangle test (tl_dual_load) while wf_trace
// keeps the fetch inside each branch (fewer live registers at 64 VGPRs).
// t0 / t1 of RT:312-313 for the four children of a ray with finite 1/d: near / far planes chosen
// per ray by the load offsets (nx..fz = near x, y, z, far x, y, z); children in pairs with packed
// fp32 (v_pk_add_f32 / v_pk_mul_f32: the same IEEE operations, two at a time)
RTD void tl_qnode_t01(const TraceLane& L, const float4 nx, const float4 ny, const float4 nz, const float4 fx,
                      const float4 fy, const float4 fz, float (&t0)[4], float (&t1)[4]) {
  const v2f ox = {L.ox, L.ox}, oy = {L.oy, L.oy}, oz = {L.oz, L.oz};
  const v2f ix = {L.ix, L.ix}, iy = {L.iy, L.iy}, iz = {L.iz, L.iz};
  const v2f nx01 = (v2f{nx.x, nx.y} - ox) * ix, ny01 = (v2f{ny.x, ny.y} - oy) * iy, nz01 = (v2f{nz.x, nz.y} - oz) * iz;
  const v2f nx23 = (v2f{nx.z, nx.w} - ox) * ix, ny23 = (v2f{ny.z, ny.w} - oy) * iy, nz23 = (v2f{nz.z, nz.w} - oz) * iz;
  const v2f fx01 = (v2f{fx.x, fx.y} - ox) * ix, fy01 = (v2f{fy.x, fy.y} - oy) * iy, fz01 = (v2f{fz.x, fz.y} - oz) * iz;
  const v2f fx23 = (v2f{fx.z, fx.w} - ox) * ix, fy23 = (v2f{fy.z, fy.w} - oy) * iy, fz23 = (v2f{fz.z, fz.w} - oz) * iz;
  t0[0] = max_(nx01.x, max_(ny01.x, nz01.x)); t1[0] = min_(fx01.x, min_(fy01.x, fz01.x));
  t0[1] = max_(nx01.y, max_(ny01.y, nz01.y)); t1[1] = min_(fx01.y, min_(fy01.y, fz01.y));
  t0[2] = max_(nx23.x, max_(ny23.x, nz23.x)); t1[2] = min_(fx23.x, min_(fy23.x, fz23.x));
  t0[3] = max_(nx23.y, max_(ny23.y, nz23.y)); t1[3] = min_(fx23.y, min_(fy23.y, fz23.y));
}
// t0 / t1 of RT:312-313 for the four children; the box is hit iff t1 >= t0 && t1 > 0, which is
// exactly hitAABB(...) > 0 (RT:315); survivors get their entry t0 as sort key
RTD void tl_qnode_keys(const TraceLane& L, bool cull, float cull_eps, const int4 rf, const float4 p0, const float4 p1,
                       const float4 p2, const float4 p3, const float4 p4, const float4 p5, float (&k)[4], int (&r)[4]) {
  const float lim = cull ? L.limit(cull_eps) : __int_as_float(0x7f800000);
  auto keep = [&](int c, float t0, float t1, int ref) {
    const bool ok = t1 >= t0 && t1 > 0.0f && (!cull || !(t0 > lim));
    k[c] = ok ? t0 : __int_as_float(0x7f800000);
    r[c] = ok ? ref : Q_EMPTY;
  };
  if (L.finite) {
    float t0[4], t1[4];
    tl_qnode_t01(L, p0, p1, p2, p3, p4, p5, t0, t1);
    keep(0, t0[0], t1[0], rf.x);
    keep(1, t0[1], t1[1], rf.y);
    keep(2, t0[2], t1[2], rf.z);
    keep(3, t0[3], t1[3], rf.w);
  } else {  // a direction component is exactly 0: the literal slab (0 * inf -> NaN cases);
            // p0..p5 = lo x, y, z, hi x, y, z
    const float4 lx = p0, ly = p1, lz = p2, hx = p3, hy = p4, hz = p5;
    // (the per-axis min / max of the literal slab would make an empty slot's inverted box look
    // infinite, so an empty slot is a miss by its ref)
    auto generic = [&](int c, float ax, float ay, float az, float bx, float by, float bz, int ref) {
      const f3 f = (mk3(bx, by, bz) - L.o()) * L.inv();
      const f3 n = (mk3(ax, ay, az) - L.o()) * L.inv();
      const bool empty = ref == Q_EMPTY;
      keep(c, empty ? __int_as_float(0x7f800000) : max_(min_(f.x, n.x), max_(min_(f.y, n.y), min_(f.z, n.z))),
           empty ? __int_as_float(0xff800000) : min_(max_(f.x, n.x), min_(max_(f.y, n.y), max_(f.z, n.z))), ref);
    };
    generic(0, lx.x, ly.x, lz.x, hx.x, hy.x, hz.x, rf.x);
    generic(1, lx.y, ly.y, lz.y, hx.y, hy.y, hz.y, rf.y);
    generic(2, lx.z, ly.z, lz.z, hx.z, hy.z, hz.z, rf.z);
    generic(3, lx.w, ly.w, lz.w, hx.w, hy.w, hz.w, rf.w);
  }
}
// POP: pop the next subtree when no child was entered; without it the caller pops (returns true
// when it must)
// SORT = false (any-hit rays: the order of the children changes which hit ends the ray, never
// whether one is found): the lowest hit slot is entered, the others stacked in slot order
template <bool POP = true, bool SORT = true>
RTD bool tl_qnode_push(const KParams& P, TraceLane& L, const TraceStack& S, bool cull, float (&k)[4], int (&r)[4]) {
  if (!SORT) {
    const bool v0 = r[0] != Q_EMPTY, v1 = r[1] != Q_EMPTY, v2 = r[2] != Q_EMPTY, v3 = r[3] != Q_EMPTY;
    if (v3 && (v0 || v1 || v2)) tl_push(L, S, make_int2(r[3], __float_as_int(k[3])));
    if (v2 && (v0 || v1)) tl_push(L, S, make_int2(r[2], __float_as_int(k[2])));
    if (v1 && v0) tl_push(L, S, make_int2(r[1], __float_as_int(k[1])));
    L.cur = v0 ? r[0] : v1 ? r[1] : v2 ? r[2] : r[3];
    if (!POP) return L.cur == Q_EMPTY;
    L.haveCur = L.cur != Q_EMPTY || tl_pop(P, L, S, cull);
    return false;
  }
  const int n = (r[0] != Q_EMPTY) + (r[1] != Q_EMPTY) + (r[2] != Q_EMPTY) + (r[3] != Q_EMPTY);
  // valid children sort ahead of empty slots unless a valid entry key is +inf (degenerate)
  const bool ordered = !((r[0] != Q_EMPTY && !(k[0] < INFINITY)) || (r[1] != Q_EMPTY && !(k[1] < INFINITY)) ||
                         (r[2] != Q_EMPTY && !(k[2] < INFINITY)) || (r[3] != Q_EMPTY && !(k[3] < INFINITY)));
  // 5-comparator sorting network on (entry, ref); empty slots (key +inf) sink to the end
#define RT_CSWAP(a, b)                                      \
  {                                                         \
    const bool sw = k[b] < k[a];                            \
    const float tk = sw ? k[b] : k[a];                      \
    k[b] = sw ? k[a] : k[b]; k[a] = tk;                     \
    const int tr = sw ? r[b] : r[a];                        \
    r[b] = sw ? r[a] : r[b]; r[a] = tr;                     \
  }
  RT_CSWAP(0, 1) RT_CSWAP(2, 3) RT_CSWAP(0, 2) RT_CSWAP(1, 3) RT_CSWAP(1, 2)
#undef RT_CSWAP
  // a +inf key can only be a valid child in degenerate cases; keep the entry count exact
  const int2 e1 = make_int2(r[1], __float_as_int(k[1])), e2 = make_int2(r[2], __float_as_int(k[2])),
             e3 = make_int2(r[3], __float_as_int(k[3]));
  if (L.sp + 3 <= S.KL && n > 0 && ordered) {
    // branch-free: the far-to-near entries 3, 2, 1 land at sp, sp+[n>=4], sp+[n>=4]+[n>=3];
    // an empty entry is overwritten by the next write, so exactly n-1 entries survive
    const int a0 = L.sp, a1 = a0 + (n >= 4), a2 = a1 + (n >= 3);
    S.lds[a0 * TL_LANES] = e3;
    S.lds[a1 * TL_LANES] = e2;
    S.lds[a2 * TL_LANES] = e1;
    L.sp += n - 1;
  } else {
    if (r[3] != Q_EMPTY) tl_push(L, S, e3);
    if (r[2] != Q_EMPTY) tl_push(L, S, e2);
    if (r[1] != Q_EMPTY) tl_push(L, S, e1);
  }
  L.cur = r[0];
  if (!POP) return r[0] == Q_EMPTY;
  L.haveCur = r[0] != Q_EMPTY || tl_pop(P, L, S, cull);
  return false;
}
template <bool POP = true, bool SORT = true>
RTD bool tl_qnode(const KParams& P, TraceLane& L, const TraceStack& S, bool cull) {
#ifdef RT_CHECK
  if ((unsigned)L.cur >= (unsigned)P.n_qnodes) {
    printf("[rt check] node %d of %d (sp %d)\n", L.cur, P.n_qnodes, L.sp);
    L.cur = 0;
  }
#endif
  const uint32_t off = (uint32_t)L.cur << 7;
  const int4 rf = ld<int4>(P.qnodes, off + 96u);
  float k[4];
  int r[4];
  if (L.finite) {
    const float4 nx = ld<float4>(P.qnodes, off + L.offNx), ny = ld<float4>(P.qnodes, off + L.offNy),
                 nz = ld<float4>(P.qnodes, off + L.offNz);
    const float4 fx = ld<float4>(P.qnodes, off + (48 - L.offNx)), fy = ld<float4>(P.qnodes, off + (80 - L.offNy)),
                 fz = ld<float4>(P.qnodes, off + (112 - L.offNz));
    tl_qnode_keys(L, cull, P.cull_eps, rf, nx, ny, nz, fx, fy, fz, k, r);
  } else {
    const float4 lx = ld<float4>(P.qnodes, off), ly = ld<float4>(P.qnodes, off + 16u),
                 lz = ld<float4>(P.qnodes, off + 32u), hx = ld<float4>(P.qnodes, off + 48u),
                 hy = ld<float4>(P.qnodes, off + 64u), hz = ld<float4>(P.qnodes, off + 80u);
    tl_qnode_keys(L, cull, P.cull_eps, rf, lx, ly, lz, hx, hy, hz, k, r);
  }
  return tl_qnode_push<POP, SORT>(P, L, S, cull, k, r);
}
// the node fetch alone (the finisher issues it before its triangle test): rf + six planes, near /
// far for a finite 1/d, lo / hi otherwise (tl_start's offsets cover both)
struct QLoad {
  int4 rf;
  float4 p[6];
};
RTD QLoad tl_qnode_load(const KParams& P, const TraceLane& L) {
  const uint32_t off = (uint32_t)L.cur << 7;
  QLoad q;
  q.rf = ld<int4>(P.qnodes, off + 96u);
  q.p[0] = ld<float4>(P.qnodes, off + L.offNx);
  q.p[1] = ld<float4>(P.qnodes, off + L.offNy);
  q.p[2] = ld<float4>(P.qnodes, off + L.offNz);
  q.p[3] = ld<float4>(P.qnodes, off + (48 - L.offNx));
  q.p[4] = ld<float4>(P.qnodes, off + (80 - L.offNy));
  q.p[5] = ld<float4>(P.qnodes, off + (112 - L.offNz));
  return q;
}
RTD bool tl_qnode_calc(const KParams& P, TraceLane& L, const TraceStack& S, bool cull, const QLoad& q) {
  float k[4];
  int r[4];
  tl_qnode_keys(L, cull, P.cull_eps, q.rf, q.p[0], q.p[1], q.p[2], q.p[3], q.p[4], q.p[5], k, r);
  return tl_qnode_push<false>(P, L, S, cull, k, r);  // the caller pops
}

// start a ray on a lane whose origin, direction and anyhit are set: 1/d, plane offsets, root
template <bool WIDE>
RTD void tl_start(const KParams& P, TraceLane& L) {
  L.ix = 1.0f / L.dx; L.iy = 1.0f / L.dy; L.iz = 1.0f / L.dz;
  // finite 1/d: per axis (lo-o)*inv <= (hi-o)*inv exactly when inv > 0 (rounding is
  // monotone), so the slab min/max of RT:309-310 is a fixed choice of plane per ray
  L.finite = fabs_(L.ix) < INFINITY && fabs_(L.iy) < INFINITY && fabs_(L.iz) < INFINITY;
  // (a ray with a zero direction component reads lo / hi: offsets 0, 16, 32 / 48, 64, 80)
  L.offNx = (L.ix > 0.0f || !L.finite) ? 0 : 48;
  L.offNy = (L.iy > 0.0f || !L.finite) ? 16 : 64;
  L.offNz = (L.iz > 0.0f || !L.finite) ? 32 : 80;
  L.set_best(INF, P.cull_eps);
  L.besttri = -1;
  L.bestt = 0.0f;
  L.sp = 0;
  L.cur = WIDE ? P.qroot : P.root;
  L.haveCur = true;
  L.tri_i = L.tri_end = 0;
}

// one dual-cursor step of a lane's ray: one triangle of the current leaf and one
// node; true when the ray is finished (stack empty and leaf done, or an any-hit found)
template <bool WIDE>
RTD bool tl_dual_step(const KParams& P, TraceLane& L, const TraceStack& TS, bool cull) {
  bool finished = false;
  if (L.tri_i < L.tri_end) {
    if (tl_triangle<WIDE>(P, L, L.tri_i++) && L.anyhit) {
      finished = true;
      L.tri_end = L.tri_i;
    }
  }
  if (!finished && L.haveCur) {
    if (ref_is_leaf(L.cur)) {
      if (L.tri_i >= L.tri_end) {  // triangle cursor free: take the leaf, move on
        L.tri_i = leaf_first(L.cur);
        L.tri_end = L.tri_i + leaf_count(L.cur);
        L.haveCur = tl_pop(P, L, TS, cull);
      }
    } else if (WIDE) {
      tl_qnode(P, L, TS, cull);
    } else {
      tl_node(P, L, TS, cull);
    }
  }
  return finished || (!L.haveCur && L.tri_i >= L.tri_end);
}

// Fetch half of one dual step: the triangle's 48 B and the node's 112 B of lane ray L (when it
// has them to do), before either test
#ifndef RT_FINISH_TRI_PAIR  // the finisher fetches and tests two triangles of a leaf per step
#define RT_FINISH_TRI_PAIR 1
#endif
struct DualLoad {
  float4 A, B, Cc, A2, B2, C2;
  QLoad q;
  bool doTri, doTri2, doNode;
};
template <bool PAIR = RT_FINISH_TRI_PAIR>
RTD DualLoad tl_dual_load(const KParams& P, const TraceLane& L, bool active) {
  DualLoad d;
  d.doTri = active && L.tri_i < L.tri_end;
  d.doNode = active && L.haveCur && !ref_is_leaf(L.cur);
  d.doTri2 = PAIR && d.doTri && L.tri_i + 1 < L.tri_end;
  d.A = d.B = d.Cc = d.A2 = d.B2 = d.C2 = make_float4(0, 0, 0, 0);
  if (d.doTri) {
    const uint32_t off = (uint32_t)L.tri_i * 48u;
    d.A = ld<float4>(P.trx, off);
    d.B = ld<float4>(P.trx, off + 16u);
    d.Cc = ld<float4>(P.trx, off + 32u);
  }
  if (d.doTri2) {
    const uint32_t off = (uint32_t)L.tri_i * 48u + 48u;
    d.A2 = ld<float4>(P.trx, off);
    d.B2 = ld<float4>(P.trx, off + 16u);
    d.C2 = ld<float4>(P.trx, off + 32u);
  }
  if (d.doNode) d.q = tl_qnode_load(P, L);
  return d;
}
// ... and the test half: the same steps as tl_dual_step (4-wide tree); true when the ray is done
RTD bool tl_dual_calc(const KParams& P, TraceLane& L, const TraceStack& TS, bool cull, const DualLoad& d) {
  bool finished = false;
  if (d.doTri) {  // (the pair in index order, each test against the best after the one before)
    if (tl_triangle_calc<true>(P, L, L.tri_i, d.A, d.B, d.Cc) && L.anyhit) finished = true;
    L.tri_i++;
    if (!finished && d.doTri2) {
      if (tl_triangle_calc<true>(P, L, L.tri_i, d.A2, d.B2, d.C2) && L.anyhit) finished = true;
      L.tri_i++;
    }
    if (finished) L.tri_end = L.tri_i;
  }
  bool needPop = false;  // one pop site (as in wf_trace)
  if (!finished && L.haveCur) {
    if (!d.doNode) {  // a leaf: taken once the triangle cursor is free
      if (L.tri_i >= L.tri_end) {
        L.tri_i = leaf_first(L.cur);
        L.tri_end = L.tri_i + leaf_count(L.cur);
        needPop = true;
      }
    } else {
      needPop = tl_qnode_calc(P, L, TS, cull, d.q);
    }
  }
  if (needPop) L.haveCur = tl_pop(P, L, TS, cull);
  return finished || (!L.haveCur && L.tri_i >= L.tri_end);
}
// the finisher's traversal step: both fetches first, then both tests, one memory round trip per
// step instead of two.  It holds ~40 more values in flight than wf_trace's 64-VGPR budget allows
// (issuing both together there cost 7% at 5 instead of 8 waves/SIMD); the finisher's latency-bound
// waves have registers to spare (C3 1080p single frames -2.2%).  The binary tree keeps tl_dual_step.
template <bool WIDE>
RTD bool tl_step_prefetch(const KParams& P, TraceLane& L, const TraceStack& TS, bool cull) {
  if (!WIDE) return tl_dual_step<WIDE>(P, L, TS, cull);
  return tl_dual_calc(P, L, TS, cull, tl_dual_load(P, L, true));
}

// ---- cooperative traversal: four lanes per ray (wf_finish's drained waves, RT_FINISH_COOP).
// The four lanes of a quad hold identical copies of one path's state (ray, best hit, cursors,
// stack) and make identical decisions; only two parts are split: lane c of the quad tests child
// box c of a 4-wide node, and triangle tri_i + c of the current leaf.  The quad's results are
// exchanged with DPP quad broadcasts, so each lane then runs the usual push (its own stack copy)
// and merges the four triangle candidates in index order with the sequential rules (dist <= best,
// exact ties by tie_wins, an any-hit ray stops at its first accepted triangle): the same closest
// hit as testing them one after the other.
// lane K of each group of G (2 or 4) consecutive lanes, to the whole group (DPP quad_perm)
template <int G, int K>
RTD int grp_bcast(int x) {
  constexpr int a = K, b = (G == 4) ? K : K + 2;
  return __builtin_amdgcn_update_dpp(0, x, a | a << 2 | b << 4 | b << 6, 0xf, 0xf, false);
}
template <int G, int K>
RTD float grp_bcast(float x) {
  return __int_as_float(grp_bcast<G, K>(__float_as_int(x)));
}
// child j's box of node L.cur with the operations of tl_qnode_keys: its sort key and ref (+inf /
// Q_EMPTY when missed or culled)
RTD void coop_box(const KParams& P, const TraceLane& L, int j, bool cull, float lim, float& key, int& rr) {
  const uint32_t off = ((uint32_t)L.cur << 7) + 4u * (uint32_t)j;
  const int ref = ld<int>(P.qnodes, off + 96u);
  float t0, t1;
  if (L.finite) {  // tl_qnode_t01 for one child
    const float nx = ld<float>(P.qnodes, off + L.offNx), ny = ld<float>(P.qnodes, off + L.offNy),
                nz = ld<float>(P.qnodes, off + L.offNz);
    const float fx = ld<float>(P.qnodes, off + (48 - L.offNx)), fy = ld<float>(P.qnodes, off + (80 - L.offNy)),
                fz = ld<float>(P.qnodes, off + (112 - L.offNz));
    t0 = max_((nx - L.ox) * L.ix, max_((ny - L.oy) * L.iy, (nz - L.oz) * L.iz));
    t1 = min_((fx - L.ox) * L.ix, min_((fy - L.oy) * L.iy, (fz - L.oz) * L.iz));
  } else {  // the literal slab (tl_qnode_keys' generic case)
    const f3 n = (mk3(ld<float>(P.qnodes, off), ld<float>(P.qnodes, off + 16u), ld<float>(P.qnodes, off + 32u)) - L.o()) * L.inv();
    const f3 f = (mk3(ld<float>(P.qnodes, off + 48u), ld<float>(P.qnodes, off + 64u), ld<float>(P.qnodes, off + 80u)) - L.o()) * L.inv();
    const bool empty = ref == Q_EMPTY;
    t0 = empty ? __int_as_float(0x7f800000) : max_(min_(f.x, n.x), max_(min_(f.y, n.y), min_(f.z, n.z)));
    t1 = empty ? __int_as_float(0xff800000) : min_(max_(f.x, n.x), min_(max_(f.y, n.y), max_(f.z, n.z)));
  }
  const bool ok = t1 >= t0 && t1 > 0.0f && (!cull || !(t0 > lim));
  key = ok ? t0 : __int_as_float(0x7f800000);
  rr = ok ? ref : Q_EMPTY;
}
// node step: lane c of the group tests children c (and c + 2 for pairs), then every lane pushes
// all four
template <int G>
RTD bool tl_qnode_coop(const KParams& P, TraceLane& L, const TraceStack& S, bool cull, int c) {
#ifdef RT_CHECK
  if ((unsigned)L.cur >= (unsigned)P.n_qnodes) printf("[rt check] coop node %d of %d\n", L.cur, P.n_qnodes);
#endif
  const float lim = cull ? L.limit(P.cull_eps) : __int_as_float(0x7f800000);
  float ka, k[4];
  int ra, r[4];
  coop_box(P, L, c, cull, lim, ka, ra);
  k[0] = grp_bcast<G, 0>(ka); k[1] = grp_bcast<G, 1>(ka);
  r[0] = grp_bcast<G, 0>(ra); r[1] = grp_bcast<G, 1>(ra);
  if (G == 4) {
    k[2] = grp_bcast<G, 2>(ka); k[3] = grp_bcast<G, 3>(ka);
    r[2] = grp_bcast<G, 2>(ra); r[3] = grp_bcast<G, 3>(ra);
  } else {
    float kb;
    int rb;
    coop_box(P, L, c + 2, cull, lim, kb, rb);
    k[2] = grp_bcast<G, 0>(kb); k[3] = grp_bcast<G, 1>(kb);
    r[2] = grp_bcast<G, 0>(rb); r[3] = grp_bcast<G, 1>(rb);
  }
  return tl_qnode_push<false>(P, L, S, cull, k, r);
}
// triangle step: up to G triangles of the leaf at once; true when an any-hit ray is done
template <int G>
RTD bool tl_tri_coop(const KParams& P, TraceLane& L, int c) {
  const int n = min(G, L.tri_end - L.tri_i);
  const int i = L.tri_i + c;
  bool hit = false;
  float dist = 0.0f, t = 0.0f;
  if (c < n) {
#ifdef RT_CHECK
    if ((unsigned)i >= (unsigned)P.n_tri) printf("[rt check] coop triangle %d of %d\n", i, P.n_tri);
#endif
    const uint32_t o = (uint32_t)i * 48u;
    hit = tl_tri_hit<true>(P, L, i, ld<float4>(P.trx, o), ld<float4>(P.trx, o + 16u), ld<float4>(P.trx, o + 32u), dist, t);
  }
  const int h = hit ? 1 : 0;
  bool finished = false;
  int used = n;
  // triangle tri_i + q against the best after the ones before it (its hit flag: hit at <= the
  // best before the step, which is >= the current best); one candidate broadcast at a time
  auto merge = [&](int q, int hq, float dq, float tq) {
    if (finished || !hq || dq > L.best) return;
    const int iq = L.tri_i + q;
    if (dq == L.best && !(L.besttri >= 0 && tie_wins(P, L, iq, L.besttri))) return;
    L.set_best(dq, P.cull_eps);
    L.besttri = iq;
    L.bestt = tq;
    if (L.anyhit) {
      finished = true;
      used = q + 1;
    }
  };
  merge(0, grp_bcast<G, 0>(h), grp_bcast<G, 0>(dist), grp_bcast<G, 0>(t));
  merge(1, grp_bcast<G, 1>(h), grp_bcast<G, 1>(dist), grp_bcast<G, 1>(t));
  if (G == 4) {
    merge(2, grp_bcast<G, 2>(h), grp_bcast<G, 2>(dist), grp_bcast<G, 2>(t));
    merge(3, grp_bcast<G, 3>(h), grp_bcast<G, 3>(dist), grp_bcast<G, 3>(t));
  }
  L.tri_i += used;
  if (finished) L.tri_end = L.tri_i;
  return finished;
}
// one cooperative dual step (tl_dual_calc's order); true when the ray is done
template <int G>
RTD bool tl_coop_step(const KParams& P, TraceLane& L, const TraceStack& TS, bool cull, int c) {
  bool finished = false;
  if (L.tri_i < L.tri_end) finished = tl_tri_coop<G>(P, L, c);
  bool needPop = false;
  if (!finished && L.haveCur) {
    if (ref_is_leaf(L.cur)) {
      if (L.tri_i >= L.tri_end) {
        L.tri_i = leaf_first(L.cur);
        L.tri_end = L.tri_i + leaf_count(L.cur);
        needPop = true;
      }
    } else {
      needPop = tl_qnode_coop<G>(P, L, TS, cull, c);
    }
  }
  if (needPop) L.haveCur = tl_pop(P, L, TS, cull);
  return finished || (!L.haveCur && L.tri_i >= L.tri_end);
}

// Move a drained wave's live lanes (mask live, at most 64 / G) to lane groups of G: lanes
// G*g .. G*g+G-1 take the traversal state of the g-th live lane (registers by lane permutes; the LDS stack column and
// its overflow entries entry by entry, every lane reading entry j of its source before any lane
// writes entry j of its own).  Returns this lane's source (itself when its group holds no ray).
// Every lane of the wave must be active.  cap = the deepest stack of the scene's trees (KParams::
// stack_cap), which the overflow columns are sized for: a deeper scene moves its whole stacks.
template <int G>
RTD int coop_move(TraceLane& L, const TraceStack& TS, unsigned long long live, int lane, int cap) {
  const int nl = __popcll(live);
  const int g = lane / G;
  unsigned long long m = live;
  for (int j = 0; j < g && m; j++) m &= m - 1ull;
  const int src = (g < nl && m) ? (int)__builtin_ctzll(m) : lane;
  // (only the sources count: a lane that holds no ray may have no defined stack)
  const int sp_src = __shfl(L.sp, src);
  int spm = g < nl ? min(max(sp_src, 0), cap) : 0;
  for (int o = 32; o > 0; o >>= 1) spm = max(spm, __shfl_xor(spm, o));
  const uint32_t w0 = threadIdx.x & ~63u;
  for (int j = 0; j < min(spm, TS.KL); j++) {
    const int2 e = TS.lds0[j * TL_LANES + w0 + src];
    TS.lds0[j * TL_LANES + w0 + lane] = e;
  }
  for (int j = TS.KL; j < spm; j++) {
    const unsigned long long e = TS.ovf[(size_t)(j - TS.KL) * TS.ovs + w0 + src];
    TS.ovf[(size_t)(j - TS.KL) * TS.ovs + w0 + lane] = e;
  }
  L.ox = __shfl(L.ox, src); L.oy = __shfl(L.oy, src); L.oz = __shfl(L.oz, src);
  L.dx = __shfl(L.dx, src); L.dy = __shfl(L.dy, src); L.dz = __shfl(L.dz, src);
  L.ix = __shfl(L.ix, src); L.iy = __shfl(L.iy, src); L.iz = __shfl(L.iz, src);
  L.best = __shfl(L.best, src); L.bestt = __shfl(L.bestt, src); L.besttri = __shfl(L.besttri, src);
  L.lim = __shfl(L.lim, src);
  L.sp = sp_src; L.cur = __shfl(L.cur, src);
  L.tri_i = __shfl(L.tri_i, src); L.tri_end = __shfl(L.tri_end, src);
  L.offNx = __shfl(L.offNx, src); L.offNy = __shfl(L.offNy, src); L.offNz = __shfl(L.offNz, src);
  L.haveCur = __shfl((int)L.haveCur, src) != 0;
  L.anyhit = __shfl((int)L.anyhit, src) != 0;
  L.finite = __shfl((int)L.finite, src) != 0;
  return src;
}

#ifndef RT_COST_PER_RAY  // tile-cost probe: node + triangle steps of a ray, plus this per ray (shade, queues)
#define RT_COST_PER_RAY 16u
#endif
#ifndef RT_REFILL_MIN  // measured on C3 (tools/exp_ab.sh): 1 -> 5399, 8 -> 5755, 16 -> 5839, 32 -> 5645 Mrays/s;
                       // on the rebuilt tree with 512-ray claims: 8 / 16 / 24 / 32 -> -2.8% / 0 / +0.6% / -1.0%;
                       // final build: 20 / 24 / 28 -> +0.3% / 0 / -0.9%
#define RT_REFILL_MIN 20
#endif
#ifndef RT_TAIL_CHUNK  // rays per claim near the end of a pass queue (and per participating wave)
#define RT_TAIL_CHUNK 64u
#endif
#ifndef RT_GUIDED  // bulk passes: claim size = rays left in the segment (as of the wave's last claim there) / (its
                   // waves x RT_GUIDED), between RT_TAIL_CHUNK and the pool chunk (before: the pool chunk until
                   // the last grid lanes x RT_TAIL_FACTOR rays, then RT_TAIL_CHUNK).  A late 1024-ray claim of one
                   // costly pixel run held a wave long after the others had drained.  With one counter, C3 bulk
                   // 1 / 2 / 3 / 4: +0.49 / +0.88, +1.04 / +0.32 / -0.07%; N=8 rank shares 70.9 -> 69.9 ms (round 5,
                   // profiles/r05_ab_bulk_guided_claims_C3.log); one-frame passes keep static shares + 64-ray claims.
                   // Round 6, with a new segment's first claim tail-sized: 3 vs 2 at N = 1 +0.00% (5 rounds,
                   // profiles/r06_ab_guided3_C3.log), N = 8 slowest rank 65.8 -> 65.1 / 65.4 ms (4: 65.4 / 65.5;
                   // profiles/r06_rank_ab_claim_knobs_C3.log)
#define RT_GUIDED 3u
#endif
#ifndef RT_REFILL_MIN_AH  // the any-hit kernel's refill threshold (split queues): C3 12 / 20 / 28 -0.55 / 0 / +0.44%
                          // (profiles/r06_ab_split_knobs_C3.log), 28 / 36 / 44 0 / -0.17 / -0.45%, with the
                          // closest-hit kernel's 16 / 24 -0.45 / -0.05% (profiles/r06_ab_split_refill_C3.log)
#define RT_REFILL_MIN_AH 28
#endif
#ifndef RT_REFILL_MIN_SMALL  // the small passes' refill threshold: C3 1080p one-frame calls 4 / 6 / 8 / 12 / 16 vs 20:
                             // -0.5 / -0.7 / -1.1, -0.6 / -0.9, -0.5 / -0.7% back-to-back (round 5,
                             // profiles/r05_ab_single_refill_min_small_C3.log; the bulk stays at 20)
#define RT_REFILL_MIN_SMALL 8
#endif
#ifndef RT_TAIL_FACTOR  // the tail starts when fewer than grid lanes x this many rays remain
#define RT_TAIL_FACTOR 4u
#endif
#ifndef RT_STATIC_FRAC  // eighths of a mid-size pass handed out statically (0: all claimed); C3 1080p one-frame
                        // calls 5 / 6 / 7 / 8 vs 4: +0.4 / -2.9 / +1.1 / +2.7% (round 5, profiles/r05_ab_single_static_frac_C3.log)
#define RT_STATIC_FRAC 6
#endif
#ifndef RT_WAVE_TIMES
#define RT_WAVE_TIMES 0
#endif
#ifndef RT_TRACE_COOP  // wf_trace (small passes, STATIC): a drained wave with at most this many rays left
                       // moves them to four lanes each (0: off).  C3 1080p one-frame calls, with the
                       // finisher's quads: -12.7% back-to-back / -8.6% synchronised against the
                       // build without either, vs -7.6% / -1.3% for the finisher's alone; lane pairs
                       // from 32 paths in the finisher cost 2-3% (profiles/r04_ab_single_coop_trace_tails_pairs_C3.log)
#define RT_TRACE_COOP 16
#endif
#ifndef RT_RES_NT  // wf_trace writes its results with non-temporal stores (1): C3 bulk +0.45%
                   // (profiles/r04_ab_bulk_result_nt_C3.log); its HBM writes stay ~30 B per ray
                   // (scattered 4-B results and 8-B overflow-stack entries, each a partial sector)
#define RT_RES_NT 1
#endif
#ifndef RT_SHADOW_SORT  // the any-hit kernel of split queues sorts children by entry distance (1) or enters
                        // the lowest hit slot and stacks the rest (0): C3 +1.02% / +2.41% over one queue of
                        // both kinds (round 6, profiles/r06_ab_split_kinds_C3.log)
#define RT_SHADOW_SORT 0
#endif
#ifndef RT_TRACE_WPE_DUAL  // dual cursor at 8 waves/SIMD (64 VGPRs; its 8-B spill is on the refill path): +2.4%
#define RT_TRACE_WPE_DUAL 8
#endif
// CAM: the implicit camera pass (WFParams::cam_n); a separate instantiation so the secondary
// passes' kernels carry none of its registers.  STATIC: small groups' static first shares (below;
// a separate instantiation: the code alone cost the bulk's kernels 0.4%).
// KIND: 0 the pass's one queue (both kinds); with split queues (WFParams::split) 1 the
// continuations (closest hit) and 2 the shadow rays (any hit: no culling, no child sort, AH
// triangle test), each launch its own instantiation with no per-lane kind
template <bool COUNT, bool WIDE, bool CAM, bool STATIC = false, bool P1 = false, int KIND = 0>  // P1: pass 1's 16-B rays
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RT_TRACE_WPE_DUAL)))
void wf_trace(const WFParams W) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const KParams& P = W.K;
  const WFState& S = W.S;
  const int qin = W.pass & 1;
  constexpr bool AHK = KIND == 2;  // every ray of the launch is any-hit
  const unsigned int nq = CAM ? W.cam_n : AHK ? S.cnt[cqs(qin)] : S.cnt[cq(qin)];
  const int* __restrict__ Q = AHK ? S.queue_s[qin] : S.queue[qin];
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // the shade pass after us appends here
    S.cnt[cq(qin ^ 1)] = 0u;
    S.cnt[cqs(qin ^ 1)] = 0u;
    S.cnt[ca(qin ^ 1)] = 0u;
  }
  if (nq == 0u || !P.has_scene) {
    if (!P.has_scene) {  // empty scene: every ray misses (RT:346 reads a zero node)
      for (unsigned int i = blockIdx.x * blockDim.x + threadIdx.x; i < nq; i += gridDim.x * blockDim.x) {
        const int e = CAM ? (int)(i << 1) : Q[i];
        S.res[e] = -1;
      }
    }
    return;
  }
  // traversal stack: the top lds_entries entries of every lane in LDS ([entry][lane], 8-B
  // {ref, entry distance} pairs, conflict-free ds_read/write_b64), deeper entries in a global
  // overflow region ([entry][grid lane], coalesced) that only very deep stacks touch.
  TraceStack TS;
  TS.KL = P.lds_entries;
#ifdef RT_CHECK
  TS.cap = P.stack_cap;
#endif
  TS.lds0 = reinterpret_cast<int2*>(smem);
  TS.lds = TS.lds0 + threadIdx.x;
  TS.ovf = (gu64*)(P.stack_ovf) + blockIdx.x * TL_LANES;
  TS.ovs = P.ovf_lanes;
  // (an any-hit ray's best is +inf until the hit that ends it: nothing to cull)
  const bool cull = !AHK && (P.flags & RT_FLAG_NO_CULL) == 0;

  bool busy = false;
  bool coop = false;  // RT_TRACE_COOP: four lanes per ray (wave-uniform)
  // per-wave pool of queue slots [pool_next, pool_end), refilled 64 at a time (wave-uniform)
  unsigned int pool_next = 0, pool_end = 0;
  const unsigned int tail_rays = gridDim.x * TL_LANES * RT_TAIL_FACTOR;
  // only as many waves as the queue can feed take part: every claim is an atomic on one word,
  // and thousands of empty-handed claims in a small late pass serialise at that address
  const unsigned int wave_id = blockIdx.x * (TL_LANES / 64) + (threadIdx.x >> 6);
  const unsigned int part_waves = min(gridDim.x * (TL_LANES / 64), (nq + RT_TAIL_CHUNK - 1u) / RT_TAIL_CHUNK);
  bool drained = wave_id >= part_waves;
  // a pass smaller than the tail threshold would be claimed entirely in 64-ray chunks, and a
  // single counter serves only ~90 claims/us (a 1080p frame's first passes: 16 K - 28 K claims);
  // so in small groups (STATIC: one frame per call) each participating wave first takes
  // a static share of RT_STATIC_FRAC/8 of the queue and only the rest is claimed dynamically
  // (C3 1080p single frames: 3.97 -> 3.68 ms; the bulk's late passes lost 0.4% with it)
  const unsigned int static_per = (STATIC && RT_STATIC_FRAC > 0 && nq <= tail_rays)
      ? (unsigned int)((unsigned long long)nq * RT_STATIC_FRAC / 8u / part_waves) : 0u;
  const unsigned int static_total = static_per * part_waves;
  if (STATIC && !drained) {
    pool_next = wave_id * static_per;
    pool_end = pool_next + static_per;
  }
  // The pass's queue in 8 segments, each claimed through its own counter (S.cnt[xcnt(s)], a cache
  // line each); a wave starts on segment blockIdx % 8 (its XCD) and moves on when a segment is
  // exhausted, drained after 8 empty segments.  Bulk passes: C3 -0.13% (noise), N=8 rank shares
  // 70.1 / 70.4 -> 69.4 / 69.7 ms (profiles/r05_ab_bulk_segment_claims_C3.log,
  // profiles/r05_rank_sim_segment_claims/); the small passes after their static shares: C3 1080p
  // one-frame calls -1.3% (profiles/r05_ab_single_segment_claims_C3.log); round 5, both against
  // one claim counter for the pass
  unsigned int seg = blockIdx.x & 7u, seg_tries = 0, seg_seen = 0;
  const unsigned int seg_waves = max(1u, part_waves / 8u);
  const int lane = (int)(threadIdx.x & 63);
  int entry = 0;
  TraceLane L;
  L.ox = L.oy = L.oz = L.dx = L.dy = L.dz = L.ix = L.iy = L.iz = 0.0f;
  L.best = INF; L.bestt = 0.0f; L.besttri = -1; L.lim = INF;
  L.sp = L.cur = L.tri_i = L.tri_end = 0;
  L.haveCur = L.anyhit = false;
  unsigned long long v_int = 0, v_leaf = 0, v_tri = 0, v_iter = 0;
  unsigned int ray_steps = 0, ray_steps_max = 0;  // COUNT: node + triangle steps of the lane's ray
  unsigned long long v_itN = 0, v_itT = 0, v_itO = 0, v_park = 0, v_busyO = 0;  // COUNT: lane utilisation
  unsigned long long v_rays = 0, v_ovf = 0;  // COUNT: rays, overflow-column pushes
  unsigned long long v_q[6] = {0, 0, 0, 0, 0, 0};  // COUNT: node visits by breadth-first index
  // RT_WAVE_TIMES (measurement builds): the release kernels log each wave's start / end / iterations
  // / rays into P.wave_log too (RT_DEBUG_PASSES), as the COUNT kernels do
  constexpr bool WT = COUNT || RT_WAVE_TIMES;
  const unsigned long long t_start = WT ? wall_clock64() : 0ull;
  const unsigned long long c_start = WT ? clock64() : 0ull;  // shader clock (s_memtime)

  while (true) {
    if (WT) v_iter++;
    // ---- refill idle lanes from the wave's pool.  A single atomic address sustains only ~90
    // atomics/us, so the pool is claimed in big chunks (P.pool_chunk rays per atomic) while plenty
    // of rays remain and in smaller ones towards the end, so the last rays still spread over all
    // waves: in the bulk passes from 8 queue segments by guided self-scheduling (RT_GUIDED), in the
    // small passes from the segments after their static shares, in 64s.
    const unsigned long long idle = __ballot(!busy);
    // refill once RT_REFILL_MIN lanes are idle (or the whole wave): the refill code runs for the
    // idle lanes only, so doing it every iteration for one or two lanes costs more issue slots
    // than the lanes it brings back
    if (idle && !drained && (__popcll(idle) >= (STATIC ? RT_REFILL_MIN_SMALL : AHK ? RT_REFILL_MIN_AH : RT_REFILL_MIN) || idle == __ballot(true))) {
      if (pool_next >= pool_end) {
        while (true) {  // (wave-uniform)
          // (small passes: the segments split what the static shares leave, claimed in 64s)
          const unsigned int d0 = STATIC ? static_total : 0u, dn = nq - d0;
          const unsigned int lo = d0 + (unsigned int)((unsigned long long)dn * seg / 8u);
          const unsigned int hi = d0 + (unsigned int)((unsigned long long)dn * (seg + 1u) / 8u);
          const unsigned int left = hi - min(max(seg_seen, lo), hi);
          const unsigned int chunk = STATIC ? RT_TAIL_CHUNK
              : min((unsigned)P.pool_chunk, max(RT_TAIL_CHUNK, (left / (seg_waves * RT_GUIDED)) & ~63u));
          unsigned int b = 0;
          if (lane == 0) b = atomicAdd(&S.cnt[AHK ? xcnts(seg) : xcnt(seg)], chunk);
          b = lo + __builtin_amdgcn_readfirstlane(__shfl(b, 0));
          if (b < hi) {
            pool_next = b;
            pool_end = min(b + chunk, hi);
            seg_seen = pool_end;
            break;
          }
          if (++seg_tries >= 8u) {
            drained = true;
            break;
          }
          seg = (seg + 1u) & 7u;
          // unknown fill of the next segment (it may be nearly drained): its first claim is the
          // tail chunk, later ones are guided by the counter value that claim returned
          seg_seen = 0xFFFFFFFFu;
        }
      }
      if (!drained || pool_next < pool_end) {
        const unsigned int avail = pool_end - pool_next;
        // idle lanes below this one (v_mbcnt: no per-lane 64-bit mask kept across the loop)
        const unsigned int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
        if (!busy && rank < avail) {
          const unsigned int qi = pool_next + rank;
          if (CAM) {  // implicit camera pass: queue entry i is slot i's camera ray
            const unsigned int slot = qi;
            entry = (int)(slot << 1);
            L.anyhit = false;
            uint32_t seed_unused, frame_unused;
            const f3 d = camera_ray(P, S, slot, seed_unused, frame_unused);
            L.ox = P.pos[0]; L.oy = P.pos[1]; L.oz = P.pos[2];
            L.dx = d.x; L.dy = d.y; L.dz = d.z;
          } else {
            entry = Q[qi];
            const int path = entry >> 1;
            L.anyhit = KIND == 2 ? true : KIND == 1 ? false : (entry & 1) != 0;
            const float4 oa = L.anyhit ? S.sa[path] : S.ra[path];
            if (P1) {  // 16-B rays from pass 0
              p1_ray(S, (unsigned)W.n_frames, (unsigned)path, oa, L.ox, L.oy, L.oz);
              L.dx = oa.x; L.dy = oa.y; L.dz = oa.z;
            } else {
              const float2 ob = L.anyhit ? S.sb[path] : S.rb[path];
              L.ox = oa.x; L.oy = oa.y; L.oz = oa.z;
              L.dx = oa.w; L.dy = ob.x; L.dz = ob.y;
            }
          }
          tl_start<WIDE>(P, L);
          busy = true;
        }
        pool_next += min((unsigned int)__popcll(idle), avail);
      }
    }
    // a drained wave (queue and pool empty) with at most RT_TRACE_COOP rays left traces them with
    // four lanes each (tl_coop_step, as in wf_finish): the pass ends on its longest rays
    if (RT_TRACE_COOP && STATIC && WIDE && !coop && drained &&
        pool_next >= pool_end) {
      const unsigned long long live = __ballot(busy);
      const int nl = __popcll(live);
      if (nl > 0 && nl <= RT_TRACE_COOP) {
        coop = true;
        const int src = coop_move<4>(L, TS, live, lane, P.stack_cap);
        const int e_src = __shfl(entry, src), b_src = __shfl((int)busy, src);
        entry = e_src;
        busy = (lane >> 2) < nl && b_src != 0;
      }
    }
    if (!__any(busy)) break;
    if (COUNT) { v_itO++; if (busy) v_busyO++; }
    bool finished = false;
    if (COUNT) { v_itN++; v_itT++; }
    if (RT_TRACE_COOP && STATIC && WIDE && coop) {
      if (busy) finished = tl_coop_step<4>(P, L, TS, cull, lane & 3);
    } else if (busy) {
      if (L.tri_i < L.tri_end) {
        if (COUNT) { v_tri++; ray_steps++; }
        if (tl_triangle<WIDE, AHK>(P, L, L.tri_i++) && (AHK || (KIND == 0 && L.anyhit))) {
          finished = true;
          L.tri_end = L.tri_i;
        }
      }
      bool needPop = false;  // one pop site per iteration (leaf taken, or no child entered)
      if (!finished && L.haveCur) {
        if (ref_is_leaf(L.cur)) {
          if (L.tri_i >= L.tri_end) {  // triangle cursor free: take the leaf, move on
            if (COUNT) { v_leaf++; v_park++; }
            L.tri_i = leaf_first(L.cur);
            L.tri_end = L.tri_i + leaf_count(L.cur);
            needPop = true;
          }
        } else {
          if (COUNT) {
            v_int++; ray_steps++;
            if (WIDE) {  // node-visit histogram by breadth-first index (the LDS cache candidates)
              v_q[0] += L.cur < 1; v_q[1] += L.cur < 5; v_q[2] += L.cur < 21;
              v_q[3] += L.cur < 64; v_q[4] += L.cur < 85; v_q[5] += L.cur < 341;
            }
          }
          const int sp0 = L.sp;
          if (WIDE) needPop = tl_qnode<false, !AHK || RT_SHADOW_SORT>(P, L, TS, cull);
          else tl_node(P, L, TS, cull);
          if (COUNT) v_ovf += (unsigned)max(0, L.sp - max(sp0, TS.KL));  // entries pushed to the overflow column
        }
      }
      if (needPop) L.haveCur = tl_pop(P, L, TS, cull);
      if (!finished && !L.haveCur && L.tri_i >= L.tri_end) finished = true;
    }
    if (busy && finished) {
      if (RT_RES_NT) __builtin_nontemporal_store(L.besttri, &S.res[entry]);
      else S.res[entry] = L.besttri;
      if (COUNT) {
        if (P.tile_cost) {  // rt_tile_costs probe: traversal steps + a per-ray share for the shade
          const unsigned int w = (unsigned int)(entry >> 1) / (unsigned int)P.n_frames;
          atomicAdd(&P.tile_cost[P.cost_blocks ? w >> 6 : S.pix_acc[w] / (unsigned int)(P.tile_w * P.tile_h)],
                    (unsigned long long)(ray_steps + RT_COST_PER_RAY));
        }
        if (P.wave_log && !(P.flags & kFlagNoRayHist))  // RT_DEBUG_PASSES: steps-per-ray histogram by kind (16-step buckets)
          atomicAdd(&P.stats[32 + (L.anyhit ? 32 : 0) + (L.besttri >= 0 ? 16 : 0) + min(15u, ray_steps / 16u)], 1ull);
        ray_steps_max = max(ray_steps_max, ray_steps); ray_steps = 0;
      }
      if (WT) v_rays++;
      busy = false;
    }
  }
  if (WT && !COUNT && P.wave_log) {
    unsigned long long r = v_rays;
    for (int off = 32; off > 0; off >>= 1) r += __shfl_xor(r, off);
    if ((threadIdx.x & 63) == 0) {
      unsigned long long* w = P.wave_log + 4 * ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6));
      w[0] = t_start; w[1] = wall_clock64(); w[2] = v_iter | ((clock64() - c_start) << 20); w[3] = r;
    }
  }
  if (COUNT) {
    if (P.wave_log) {
      unsigned long long r = v_rays;
      for (int off = 32; off > 0; off >>= 1) r += __shfl_xor(r, off);
      if ((threadIdx.x & 63) == 0) {
        unsigned long long* w = P.wave_log + 4 * ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6));
        w[0] = t_start; w[1] = wall_clock64(); w[2] = v_iter | ((clock64() - c_start) << 20); w[3] = r;
      }
    }
    for (int off = 32; off > 0; off >>= 1) {
      v_int += __shfl_xor(v_int, off);
      v_leaf += __shfl_xor(v_leaf, off);
      v_tri += __shfl_xor(v_tri, off);
      v_park += __shfl_xor(v_park, off);
      v_busyO += __shfl_xor(v_busyO, off);
      v_ovf += __shfl_xor(v_ovf, off);
    }
    for (int q = 0; q < 6; q++) {
      unsigned long long x = v_q[q];
      for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
      if ((threadIdx.x & 63) == 0 && x) atomicAdd(&P.stats[22 + q], x);
    }
    if ((threadIdx.x & 63) == 0) {  // wave-uniform iteration counts + lane-sums
      atomicAdd(&P.stats[8], v_itN);
      atomicAdd(&P.stats[9], v_int + v_park);
      atomicAdd(&P.stats[10], v_itT);
      atomicAdd(&P.stats[11], v_tri);
      atomicAdd(&P.stats[12], v_itO);
      atomicAdd(&P.stats[13], v_busyO);
      atomicAdd(&P.stats[14], v_ovf);
    }
    if ((threadIdx.x & 63) == 0) {
      atomicAdd(&P.stats[2], v_int);
      atomicAdd(&P.stats[3], v_leaf);
      atomicAdd(&P.stats[4], v_tri);
      atomicAdd(&P.stats[5], v_iter);
      atomicMax(&P.stats[6], v_iter);
    }
    for (int off = 32; off > 0; off >>= 1) ray_steps_max = max(ray_steps_max, (unsigned)__shfl_xor((int)ray_steps_max, off));
    if ((threadIdx.x & 63) == 0) {
      atomicMax(&P.stats[7], (unsigned long long)ray_steps_max);
    }
  }
}

// ----------------------------------------------------------------------------- shade
// Paths per block-iteration of wf_shade = 256 x SH_SUB: the block stages its queue / active
// entries in LDS and claims global space with one atomic per list per block-iteration.
#ifndef RT_SH_SUB  // C3 on the rebuilt tree: 1 / 2 / 4 / 8 -> -1.2% / 0 / -0.9% / -1.4% (tools/ab_proc.py);
                   // final build: 3 vs 2 +0.4%; small groups (one frame per call) keep it (4: one-frame calls
                   // +6.9%, round 4: fewer blocks for their 2 M-path passes)
#define RT_SH_SUB 3
#endif
#ifndef RT_SH_SUB_BULK  // the bulk's shade launches (groups above the finisher's slot budget): round 5, C3
                        // 2 / 4 vs 3: -1.26 / +0.55%; 4 / 5 / 6 / 7 / 8: +0.40 / +0.74 / +1.02, +1.16 / +1.22 /
                        // +1.45% (profiles/r05_ab_bulk_shade_sub_C3.log; 10: 149 VGPRs, 3 waves/SIMD)
#define RT_SH_SUB_BULK 8
#endif
constexpr int SH_KEYS = 2;  // 0: no continuation hit (env / end of path); 1: a continuation hit

// what a path's shade iteration will run: the cheap end-of-path / env branch or a bounce on
// the hit material
RTD int shade_key(const KParams& P, const WFState& S, int path) {
  const uint32_t flags = S.s5[path].y & 0xffu;
  const int t = S.res[2 * path];
  if (!(flags & PF_CONT) || t < 0) return 0;
  return 1;
}
#ifndef RT_SHADE_WPE  // 4 waves/SIMD (<= 128 VGPRs, 12 B/lane spill): shade -8% vs the natural 3
#define RT_SHADE_WPE 4
#endif
#ifndef RT_SH_SUB_CAM  // the bulk camera pass's shade (wf_shade<..., CAM>): 6 / 4 vs 8 -0.22 / -0.53% (C3 bulk,
                       // round 5, profiles/r05_ab_bulk_cam_shade_sub_C3.log)
#define RT_SH_SUB_CAM RT_SH_SUB_BULK
#endif
constexpr int SH_SUB = RT_SH_SUB, SH_SUB_BULK = RT_SH_SUB_BULK, SH_SUB_CAM = RT_SH_SUB_CAM;

// One path's shade step (the body of wf_shade, shared with wf_finish): consume the traced results
// of the current bounce, sample the next one, write the state back and return the rays to queue.
// camPass: the implicit camera pass (state built from the slot); loadPrev: the path has state
// from an earlier pass (every pass but 0).
struct ShadeOut {
  bool qShadow, qCont;
};
// The closest hit's geometry (RT:265, RT:1519-1527): t, side, hit point, interpolated normal and
// material of triangle `tri` on ray (ro, rd) -- tl_triangle_calc's operations on the same ray and
// triangle.
struct HitGeom {
  float t;
  bool inside;
  f3 Pp, Ns;
  int nmat;
};
// The six texels come from the triangle's 128-B hit record (KParams::hrec: one cache line) rather
// than from tri and trin, whose 48-B records straddle a line boundary 37% of the time (2.7 lines
// per hit instead of 1, fetched from MALL: the continuation's triangle is a scattered access)
#ifndef RT_HREC
#define RT_HREC 1
#endif
RTD HitGeom hit_geom(const KParams& P, int tri, f3 ro, f3 rd) {
  const float4* h4 = RT_HREC ? P.hrec + 8 * tri : nullptr;
  const float4 A = RT_HREC ? h4[0] : P.tri[3 * tri], B = RT_HREC ? h4[1] : P.tri[3 * tri + 1],
               Cc = RT_HREC ? h4[2] : P.tri[3 * tri + 2];
  const float4 N1 = RT_HREC ? h4[3] : P.trin[3 * tri], N2 = RT_HREC ? h4[4] : P.trin[3 * tri + 1],
               N3 = RT_HREC ? h4[5] : P.trin[3 * tri + 2];
  const f3 p1 = xyz(A), p2 = xyz(B), p3 = xyz(Cc);
  const f3 ng = mk3(A.w, B.w, Cc.w);
  HitGeom h;
  h.t = (dot(ng, p1) - dot(ro, ng)) / dot(rd, ng);
  h.inside = dot(ng, rd) > 0.0f;
  const f3 Pp = ro + rd * h.t;
  const float alpha = (-(Pp.x - p2.x) * (p3.y - p2.y) + (Pp.y - p2.y) * (p3.x - p2.x)) /
                      (-(p1.x - p2.x) * (p3.y - p2.y) + (p1.y - p2.y) * (p3.x - p2.x) + 1e-7f);
  const float beta = (-(Pp.x - p3.x) * (p1.y - p3.y) + (Pp.y - p3.y) * (p1.x - p3.x)) /
                     (-(p2.x - p3.x) * (p1.y - p3.y) + (p2.y - p3.y) * (p1.x - p3.x) + 1e-7f);
  const float gama = 1.0f - alpha - beta;
  h.Pp = Pp;
  h.Ns = normalize(alpha * xyz(N1) + beta * xyz(N2) + gama * xyz(N3));
  h.nmat = __float_as_int(N1.w);
  return h;
}

// Camera pass of the bulk groups (wf_shade<..., CAM>, RT_CAM_SHADE in rt_render.hip): a
// block-iteration's paths are a few pixels' frames, and every frame of a pixel shades the same
// camera hit (R6: no jitter).  What depends only on that hit -- geometry, emission, the BSDF frame,
// or the environment colour of a miss -- is computed once per pixel into LDS (kCamRec float4) by
// cam_rec and read by the frames' lanes (same functions on the same values: the same bits), with
// the terms of the BSDF calls that depend on V and the material alone (v_terms: DisneySample's
// lobe weights, the VNDF frame, the V-side Fresnel and masking terms).  Every frame of a pixel has
// the record's trace result (the same ray, and a closest hit that is a function of the ray:
// RT_CHECK reports any frame that does not).  The other instantiations carry none of it (a
// runtime record path in them cost the later passes' shades 2 ms per 256-frame group).
constexpr int kCamRec = 11;  // [0..6] the hit, [7..10] v_terms
RTD void cam_rec(const WFParams& W, const Env& E, unsigned int w, float4* rec) {
  const KParams& P = W.K;
  const WFState& S = W.S;
  const unsigned int path0 = w * (unsigned)W.n_frames;  // frame 0 of work item w
  int r = S.res[2 * path0];
  const f3 ro = mk3(P.pos[0], P.pos[1], P.pos[2]), rd = xyz(S.cam[w]);
#ifdef RT_CHECK
  if (r >= P.n_tri) r = -1;  // (shade_path reports it)
#endif
  if (r >= 0) {
    const HitGeom h = hit_geom(P, r, ro, rd);
    const f3 hN = h.inside ? -h.Ns : h.Ns;
    const Mat m = load_mat(P.mats, h.nmat);
    const BsdfFrame BF = bsdf_frame(m, -rd, hN);
    const f3 Le0 = xyz(P.mats[8 * h.nmat]);
    rec[0] = make_float4(h.Pp.x, h.Pp.y, h.Pp.z, h.t - 0.00001f);
    rec[1] = make_float4(hN.x, hN.y, hN.z, __int_as_float(r));
    rec[2] = make_float4(Le0.x, Le0.y, Le0.z, __int_as_float(h.nmat));
    rec[3] = make_float4(BF.eta, BF.T.x, BF.T.y, BF.T.z);
    rec[4] = make_float4(BF.B.x, BF.B.y, BF.B.z, BF.V.x);
    rec[5] = make_float4(BF.V.y, BF.V.z, BF.specCol.x, BF.specCol.y);
    rec[6] = make_float4(BF.specCol.z, BF.sheenCol.x, BF.sheenCol.y, BF.sheenCol.z);
    v_terms(BF, m, rec + 7);
  } else {
    const f3 env = P.enable_env ? hdrColor(E, rd) * E.intensity : getDefaultSkyColor(rd.y);
    rec[1] = make_float4(0.0f, 0.0f, 0.0f, __int_as_float(r));
    rec[2] = make_float4(env.x, env.y, env.z, 0.0f);
  }
}
RTD BsdfFrame rec_frame(const float4* rec) {
  const float4 q3 = rec[3], q4 = rec[4], q5 = rec[5], q6 = rec[6];
  BsdfFrame F;
  F.eta = q3.x;
  F.T = mk3(q3.y, q3.z, q3.w);
  F.B = mk3(q4.x, q4.y, q4.z);
  F.V = mk3(q4.w, q5.x, q5.y);
  F.specCol = mk3(q5.z, q5.w, q6.x);
  F.sheenCol = mk3(q6.y, q6.z, q6.w);
  return F;
}

// CAMK: the camera pass of wf_shade<..., CAM> (every path's hit from its pixel's record)
template <bool BSDF, bool FUSE = false, bool CAMK = false>  // FUSE: W.fuse_blend is honoured (one-frame pixel groups)
RTD ShadeOut shade_path(const WFParams& W, const Env& E, int path, bool live, bool camPass, bool loadPrev,
                        unsigned long long& nsamples, const float4* rec = nullptr) {
  const KParams& P = W.K;
  const WFState& S = W.S;
  bool doFinish = false, doBounce = false;
  bool qShadow = false, qCont = false;
  f3 fin = splat(0.0f);
  float4 a0 = make_float4(0, 0, 0, 0), a1 = a0, a2 = a0, a3 = a0, a4 = a0;
  uint4 a5 = make_uint4(0, 0, 0, 0);
  f3 hist = splat(1.0f), Lo = splat(0.0f), Le0 = splat(0.0f), evf = splat(0.0f);
  float evp = 0.0f;
  uint32_t wseed = 0, bounce = 0, flags = 0, frame = 0;
  f3 hP = splat(0.0f), hN = splat(0.0f), hV = splat(0.0f);
  float hDist = 0.0f;
  int mat = 0;
  constexpr bool useRec = CAMK;  // camera pass of wf_shade<..., CAM>: this path's hit is its pixel's record (cam_rec)
  if (live) {
    float4 cam_d = make_float4(0, 0, 0, 0);
    if (camPass) {  // implicit camera pass: the state a camera path starts with
      uint32_t cseed, cframe;
      const f3 d = camera_ray(P, S, (unsigned)path, cseed, cframe);
      a5 = make_uint4(cseed, 0u, PF_CONT | PF_CAMERA, cframe);
      cam_d = make_float4(d.x, d.y, d.z, 0.0f);
    } else {
      const uint2 p5 = S.s5[path];
      const unsigned int nfr = (unsigned int)W.n_frames;
      a5 = make_uint4(p5.x, p5.y >> 8, p5.y & 0xffu, (unsigned int)path % nfr);
    }
    // every load of the path's state issues at once: camera paths exist only in pass 0 (a
    // uniform test), so no load waits for the flags; the flags still decide what is used
    int rsh = 0;
    if (loadPrev) {
      a0 = S.s0[path]; a2 = S.s2[path];
      rsh = S.res[2 * path + 1];
      // (PF_ZLO) a path whose Lo and Le0 are +0 (every path after a non-emissive camera hit, whose
      // NEE is still pending) skips the s1 row and, without a shadow ray, the s3 row
      if (!(a5.z & PF_ZLO)) {
        a1 = S.s1[path];
        a3 = S.s3[path];
      } else if (a5.z & PF_SHADOW) {
        a3 = S.s3[path];
      }
    }
    const int rc0 = S.res[2 * path];
#ifdef RT_CHECK
    if (CAMK && __float_as_int(rec[1].w) != rc0)
      printf("[rt check] camera record: path %d result %d, record %d\n", path, rc0, __float_as_int(rec[1].w));
#endif
    float4 oo0, dd0;
    if (camPass) {
      oo0 = make_float4(P.pos[0], P.pos[1], P.pos[2], 0.0f);
      dd0 = make_float4(cam_d.x, cam_d.y, cam_d.z, 0.0f);
    } else if (W.p1_compact && W.pass == 1) {  // (uniform) the continuation in pass 0's 16-B form
      const float4 ra0 = S.ra[path];
      float ox, oy, oz;
      p1_ray(S, (unsigned)W.n_frames, (unsigned)path, ra0, ox, oy, oz);
      oo0 = make_float4(ox, oy, oz, 0.0f);
      dd0 = make_float4(ra0.x, ra0.y, ra0.z, 0.0f);
    } else {
      const float4 ra0 = S.ra[path];
      const float2 rb0 = S.rb[path];
      oo0 = make_float4(ra0.x, ra0.y, ra0.z, 0.0f);
      dd0 = make_float4(ra0.w, rb0.x, rb0.y, 0.0f);
    }
    wseed = a5.x; bounce = a5.y; flags = a5.z; frame = a5.w;
    if (!(flags & PF_CAMERA)) {
      hist = xyz(a0); evp = a0.w;
      Lo = xyz(a1);
      evf = xyz(a2);
      Le0 = mk3(a1.w, a2.w, 0.0f);
      Le0.z = a3.w;
      // ---- pending NEE of the previous bounce (RT:1389-1405): add if the shadow ray escaped
      if ((flags & PF_SHADOW) && rsh < 0) Lo = Lo + xyz(a3);
      // ---- pending medium-emissive term (RT:1437-1439)
      if (flags & PF_CMED) {
        a4 = S.s4[path];
        Lo = Lo + xyz(a4);
      }
    }
    if (!(flags & PF_CONT)) {  // BSDF pdf was 0 (RT:1460-1462): the path ends
      fin = Le0 + Lo;
      doFinish = true;
    } else {
      // the CAM pass branches on the record's own result (rec[1].w, written on hit and miss alike),
      // so both record branches read initialised LDS; a frame whose own result differed would be
      // reported by the RT_CHECK build above (none is: every frame traces the same camera ray, R6)
      const int r = useRec ? __float_as_int(rec[1].w) : rc0;
      const float4 oo = oo0, dd = dd0;
      const f3 ro = xyz(oo), rd = xyz(dd);
      if (useRec && r >= 0) {  // the pixel's camera hit from the record (cam_rec)
        const float4 q0 = rec[0], q1 = rec[1], q2 = rec[2];
        Le0 = xyz(q2);
        hP = xyz(q0);
        if (W.p1_compact && frame == 0u) S.org[(unsigned)path / (unsigned)W.n_frames] = make_float4(q0.x, q0.y, q0.z, 0.0f);
        hN = xyz(q1);
        hV = rd;
        hDist = q0.w;
        mat = __float_as_int(q2.w);
        if (0 < P.max_bounce) doBounce = true;
        else { fin = Le0 + Lo; doFinish = true; }
      } else if (useRec) {
        fin = xyz(rec[2]);
        doFinish = true;
      } else if (r >= 0) {
        int tri = r;
#ifdef RT_CHECK
        if (tri >= P.n_tri) {
          printf("[rt check] shade: path %d pass %d result triangle %d of %d\n", path, W.pass, tri, P.n_tri);
          tri = 0;
        }
#endif
        const HitGeom hg = hit_geom(P, tri, ro, rd);
        const float t = hg.t;
        const bool inside = hg.inside;
        const f3 Pp = hg.Pp, Ns = hg.Ns;
        const int nmat = hg.nmat;
        if (flags & PF_CAMERA) {  // RT:1541-1544
          Le0 = xyz(P.mats[8 * nmat]);
          Lo = splat(0.0f);
          hist = splat(1.0f);
          bounce = 0;
        } else if (BSDF) {  // RT:1509-1510
          const f3 Le = xyz(P.mats[8 * nmat]);
          Lo = Lo + hist * Le * evf / evp;
          bounce++;
        } else {  // BRDF mode RT:1362-1364 (evf = f_r, evp = pdf_brdf, s4.x = N.L)
          const f3 Le = xyz(P.mats[8 * nmat]);
          Lo = Lo + hist * Le * evf * fabs_(S.s4[path].x) / evp;
          bounce++;
        }
        hP = Pp;
        // pass 0: frame 0 of each pixel records the camera hit point, the origin of every frame's
        // next rays (WFState::org)
        if (camPass && W.p1_compact && frame == 0u) S.org[(unsigned)path / (unsigned)W.n_frames] = make_float4(Pp.x, Pp.y, Pp.z, 0.0f);
        hN = inside ? -Ns : Ns;
        hV = rd;
        hDist = t - 0.00001f;
        mat = nmat;
        if ((int)bounce < P.max_bounce) doBounce = true;
        else { fin = Le0 + Lo; doFinish = true; }
      } else if (flags & PF_CAMERA) {  // RT:1532-1539
        fin = P.enable_env ? hdrColor(E, rd) * E.intensity : getDefaultSkyColor(rd.y);
        doFinish = true;
      } else if (!BSDF) {  // BRDF mode RT:1345-1359
        const float aNdotL = fabs_(S.s4[path].x);
        if (P.enable_env) {
          f3 skyColor;
          float pdf_light;
          hdrColorPdf(E, rd, skyColor, pdf_light);
          skyColor = skyColor * E.intensity;
          const float mis_weight = misMixWeight(evp, pdf_light);
          Lo = Lo + mis_weight * hist * skyColor * evf * aNdotL / evp;
        } else {
          const f3 skyColor = getDefaultSkyColor(rd.y);
          Lo = Lo + hist * skyColor * evf * aNdotL / evp;
        }
        fin = Le0 + Lo;
        doFinish = true;
      } else {  // RT:1483-1506
        if (P.enable_env) {
          f3 light_fr;
          float light_pdf;
          hdrColorPdf(E, rd, light_fr, light_pdf);
          light_fr = light_fr * E.intensity;
          float mis_weight = misMixWeight(evp, light_pdf);
          if (!P.enable_mis) mis_weight = 1.0f;
          if (!(flags & PF_MEDIUM)) Lo = Lo + mis_weight * hist * light_fr * evf / evp;
          else Lo = Lo + hist * light_fr * evf / light_pdf;
        } else {
          const f3 light_fr = getDefaultSkyColor(rd.y);
          Lo = Lo + hist * light_fr * evf / evp;
        }
        fin = Le0 + Lo;
        doFinish = true;
      }
    }
  }

  // ------------------------------------------------------------- next bounce
  f3 cnee = splat(0.0f), cmed = splat(0.0f);
  uint32_t nflags = 0;
  f3 contO = splat(0.0f), contD = splat(0.0f), shO = splat(0.0f), shD = splat(0.0f);
  float contS = 0.0f;  // the continuation's scattering distance (its origin = hit point + hV * contS)
  float bNdotL = 0.0f;  // BRDF mode: N.L of the sampled direction (RT:1336)
  if (doBounce && !BSDF) {  // shadingImportanceSampling_BRDF, one iteration (RT:1296-1365)
    const Mat m = load_mat(P.mats, mat);
    const f3 V = -hV, N = hN;
    const float xa = rand_(wseed);
    const float xb = rand_(wseed);
    f3 Ll, light_fr;
    float light_pdf;
    SampleHdrLight(E, xa, xb, Ll, light_fr, light_pdf);  // SampleHdr + hdrColorPdf (same bits)
    f3 T, Bt;
    getTangent(N, T, Bt);
    if (dot(N, Ll) > 0.0f) {
      light_fr = light_fr * E.intensity;
      float brdf_pdf;
      const f3 brdf_fr = BRDF_Evaluate(V, N, Ll, T, Bt, m, brdf_pdf);
      const float mis_weight = misMixWeight(light_pdf, brdf_pdf);
      cnee = mis_weight * hist * light_fr * brdf_fr * fabs_(dot(N, Ll)) / light_pdf;
      shO = hP;
      shD = Ll;
      qShadow = true;
      nflags |= PF_SHADOW;
    }
    float sx, sy;
    sobol_pair(P, frame, bounce, sx, sy);
    const float cu = rand_(wseed), cv = rand_(wseed);
    sx += cu;
    if (sx > 1) sx -= 1;
    if (sx < 0) sx += 1;
    sy += cv;
    if (sy > 1) sy -= 1;
    if (sy < 0) sy += 1;
    const float xi_3 = rand_(wseed);
    const f3 L = SampleBRDF(sx, sy, xi_3, V, N, m);
    bNdotL = dot(N, L);
    float pdf_brdf;
    const f3 f_r = BRDF_Evaluate(V, N, L, T, Bt, m, pdf_brdf);
    if (pdf_brdf > 0.0f) {
      hist = hist * (f_r * fabs_(bNdotL) / pdf_brdf);
      evf = f_r;
      evp = pdf_brdf;
      contO = hP;
      contD = L;
      qCont = true;
      nflags |= PF_CONT;
    }
    if (!qShadow && !qCont) {
      fin = Le0 + Lo;
      doFinish = true;
    }
  } else if (doBounce) {
    const Mat m = load_mat(P.mats, mat);
    const f3 V = -hV;
    const BsdfFrame BF = useRec ? rec_frame(rec) : bsdf_frame(m, V, hN);  // shared by the three BSDF calls below
    // light sample + NEE term (RT:1380-1405), evaluated now, added after the shadow ray
    const float xa = rand_(wseed);  // R24
    const float xb = rand_(wseed);
    f3 Ll, light_fr;
    float light_pdf;
    SampleHdrLight(E, xa, xb, Ll, light_fr, light_pdf);  // SampleHdr + hdrColorPdf (same bits)
    if (dot(hN, Ll) > 0.0f) {
      light_fr = light_fr * E.intensity;
      float disney_eval_pdf;
      const f3 disney_eval_fr = DisneyEval<CAMK>(BF, m, hN, Ll, disney_eval_pdf, CAMK ? rec + 7 : nullptr);
      float mis_weight = misMixWeight(light_pdf, disney_eval_pdf);
      if (!P.enable_mis) mis_weight = 1.0f;
      cnee = mis_weight * hist * light_fr * disney_eval_fr / light_pdf;
      shO = hP;
      shD = Ll;
      qShadow = true;
      nflags |= PF_SHADOW;
    }
    // BSDF sample (RT:1408-1474)
    float sx, sy;
    sobol_pair(P, frame, bounce, sx, sy);
    const float cu = rand_(wseed), cv = rand_(wseed);
    sx += cu;
    if (sx > 1) sx -= 1;
    if (sx < 0) sx += 1;
    sy += cv;
    if (sy > 1) sy -= 1;
    if (sy < 0) sy += 1;
    const float xi_3 = rand_(wseed);
    f3 L;
    float pdf;
    bool isRefract;
    const f3 fr = DisneySample<CAMK>(BF, sx, sy, xi_3, m, hN, L, pdf, isRefract, CAMK ? rec + 7 : nullptr);
    bool medS = false;
    float scatter_pdf = 0.0f;
    float transmittance = 1.0f;
    if (pdf > 0.0f) {
      if (!isRefract) {
        hist = hist * (fr / pdf);
      } else if (m.mtype == MEDIUM_ABSORB) {
        hist = hist * exp3(-(splat(1.0f) - m.mcolor) * hDist * m.mdensity);
      } else if (m.mtype == MEDIUM_EMISSIVE) {
        cmed = m.mcolor * hDist * m.mdensity * hist;
        nflags |= PF_CMED;
      } else if (m.mtype == MEDIUM_SCATTER) {
        const float scatterDist = min_(-log_(xi_3) / m.mdensity, hDist);
        medS = scatterDist < hDist;
        if (medS) {
          contS = scatterDist;
          transmittance *= exp_(-1.0f * scatterDist);
          hist = hist * (m.mcolor * transmittance);
          hP = hP + hV * scatterDist;
          const f3 scatterDir = SampleHG(V, m.manis, sx, sy);
          scatter_pdf = PhaseHG(dot(V, scatterDir), m.manis);
          L = scatterDir;
        }
      }
      evf = DisneyEval<CAMK>(BF, m, hN, L, evp, CAMK ? rec + 7 : nullptr);
      if (medS && scatter_pdf > 0.0f) {
        evp = scatter_pdf;
        evf = splat(scatter_pdf);
      }
      if (medS) nflags |= PF_MEDIUM;
      contO = hP;
      contD = L;
      qCont = true;
      nflags |= PF_CONT;
    }
    if (!qShadow && !qCont) {  // no ray left: finish now (RT:1460-1462 break)
      fin = Le0 + Lo;
      doFinish = true;
    }
  }

  // ----------------------------------------------------------- progressive blend
  if (doFinish) {  // curColor of RT:1549; blended by wf_blend in frame order
    if (FUSE && W.fuse_blend) {  // one frame: the blend of this pixel, here (same operations as wf_blend)
      const unsigned int ai = S.pix_acc[path];
      const float4 h = P.accum[ai];
      const float2 bw = P.blend_w[frame];  // {1 / n, (n - 1) / n} (wf_sobol)
      const f3 acc = bw.x * fin + bw.y * mk3(h.x, h.y, h.z);
      P.accum[ai] = make_float4(acc.x, acc.y, acc.z, 0.0f);
    } else {
      st_row(S.fin + path, make_float4(fin.x, fin.y, fin.z, 0.0f));
    }
    nsamples++;
  }

  // ------------------------------------------------------------ enqueue rays
  const bool keep = qShadow || qCont;
  if (keep) {
    const bool zlo = (__float_as_uint(Lo.x) | __float_as_uint(Lo.y) | __float_as_uint(Lo.z) |
                                __float_as_uint(Le0.x) | __float_as_uint(Le0.y) | __float_as_uint(Le0.z)) == 0u;
    if (zlo) nflags |= PF_ZLO;
    st_row(S.s0 + path, make_float4(hist.x, hist.y, hist.z, evp));
    if (!zlo) st_row(S.s1 + path, make_float4(Lo.x, Lo.y, Lo.z, Le0.x));
    st_row(S.s2 + path, make_float4(evf.x, evf.y, evf.z, Le0.y));
    if (!zlo || qShadow) st_row(S.s3 + path, make_float4(cnee.x, cnee.y, cnee.z, Le0.z));
    if (nflags & PF_CMED) st_row(S.s4 + path, make_float4(cmed.x, cmed.y, cmed.z, 0.0f));
    if (!BSDF && qCont) st_row(S.s4 + path, make_float4(bNdotL, 0.0f, 0.0f, 0.0f));
    st_row(S.s5 + path, make_uint2(wseed, bounce << 8 | nflags));
    if (camPass && W.p1_compact) {  // (uniform) 16-B rays from the pixel's camera hit point
      if (qCont) st_row(S.ra + path, make_float4(contD.x, contD.y, contD.z, contS));
      if (qShadow) st_row(S.sa + path, make_float4(shD.x, shD.y, shD.z, 0.0f));
    } else {
      if (qCont) put_ray(S.ra, S.rb, path, contO.x, contO.y, contO.z, contD.x, contD.y, contD.z);
      if (qShadow) put_ray(S.sa, S.sb, path, shO.x, shO.y, shO.z, shD.x, shD.y, shD.z);
    }
  }
  return ShadeOut{qShadow, qCont};
}

// BSDF: enableBSDF (RT:1369 Disney integrator) or the BRDF integrator (RT:1290), one
// instantiation each so neither carries the other's registers
// CAM: the bulk groups' camera pass (>= 64 frames per group, camera-hit records), its own
// instantiation: no path state to load, so none of its registers
template <bool BSDF, bool FUSE = false, int SH_SUB = rtd::SH_SUB, bool CAM = false>  // SH_SUB: paths per thread and block-iteration
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RT_SHADE_WPE))) void wf_shade(const WFParams W) {
  __shared__ int lq[2 * 256 * SH_SUB];
  __shared__ int la[256 * SH_SUB];
  __shared__ int lsort[256 * SH_SUB];  // the block's paths, grouped by shade_key
  __shared__ unsigned int lhist[SH_KEYS], lofs[SH_KEYS];
  __shared__ unsigned int lc[6];  // queue count (shadow rays), active count, queue base, active base, continuations, (split) their base
  constexpr unsigned int kRecs = 256u * SH_SUB / 64u + 1u;  // pixels a block-iteration spans at >= 64 frames
  __shared__ float4 lrec[CAM ? kCamRec * kRecs : 1];
  // 4 waves/SIMD = 4 blocks per CU: the block's LDS must fit a quarter of the CU's 160 KB
  static_assert(4 * (2 * 256 * SH_SUB + 2 * 256 * SH_SUB) + 16 * (CAM ? kCamRec * kRecs : 1) +
                    8 * SH_KEYS + 20 <= 40960,
                "wf_shade LDS exceeds a quarter of the CU");
  const KParams& P = W.K;
  const WFState& S = W.S;
  const int in = W.pass & 1, out = in ^ 1;
  const unsigned int nfr = (unsigned int)W.n_frames;
  constexpr bool camrec = CAM;
  const unsigned int na = CAM || W.cam_n ? W.cam_n : S.cnt[ca(in)];
  const unsigned int nq_in = CAM || W.cam_n ? W.cam_n : S.cnt[cq(in)] + (W.split ? S.cnt[cqs(in)] : 0u);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    S.cnt[kCntFetch] = 0u;  // fetch counter of the next trace pass
    if (na) {
      atomicAdd(&P.stats[16], (unsigned long long)na);  // path shade steps (rt_stats.path_steps)
      if (W.pass <= 1) atomicAdd(&P.stats[18 + W.pass], (unsigned long long)na);  // pass0_steps, pass1_steps
    }
  }
  if (blockIdx.x == 0 && threadIdx.x < 16u)  // (the next trace pass's segment counters, both queues)
    S.cnt[threadIdx.x < 8u ? xcnt(threadIdx.x) : xcnts(threadIdx.x - 8u)] = 0u;
  const Env E{P.hdr, P.cache, P.light, P.hdr_w, P.hdr_h, P.hdr_res, P.env_angle, P.env_intensity};
  unsigned long long nrays = 0, nsamples = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    nrays = nq_in;  // rays traced by the pass before us
    if (W.pass == 1 && W.p1_compact && nq_in) atomicAdd(&P.stats[17], (unsigned long long)nq_in);  // rt_stats.p1_rays
  }
  for (unsigned int base = blockIdx.x * (256u * SH_SUB); base < na; base += gridDim.x * (256u * SH_SUB)) {
  // ---- group the block's paths by what they will execute (block-local counting sort in LDS):
  // divergence between a continuation that missed (env lookup) and one that hit (a full BSDF
  // bounce) or between materials otherwise idles most lanes of a wave.  Order never changes a
  // path's result.
  // Only for big secondary passes: the key loads add a dependent-latency step that small,
  // latency-bound late passes feel more than their divergence; the camera pass (lane
  // utilisation ~0.8) loses more than it gains (measured on C3, 64 frames in flight).
  const unsigned int nblk = min(256u * SH_SUB, na - base);
  if (threadIdx.x < SH_KEYS) lhist[threadIdx.x] = 0u;
  if (threadIdx.x == 0) lc[0] = lc[1] = lc[4] = 0u;
  __syncthreads();
  // sort only passes holding at least a quarter of the group's path slots (in practice pass 1,
  // whatever the per-rank pixel share)
  const bool sort_pass = !CAM && W.pass != 0 && na >= max(1u << 22, (unsigned)W.n_frames * P.n_work / 4u);
  if (!sort_pass) {  // camera pass: hit/miss divergence is low already
#pragma unroll
    for (int sub = 0; sub < SH_SUB; sub++) {
      const unsigned int j = (unsigned)sub * 256u + threadIdx.x;
      if (j < nblk) lsort[j] = CAM || W.cam_n ? (int)(base + j) : S.active[in][base + j];
    }
    if (camrec) {  // the block-iteration's pixels' camera hits, one lane each
      const unsigned int p0 = base / nfr, np = (base + nblk - 1u) / nfr - p0 + 1u;
      if (threadIdx.x < np) cam_rec(W, E, p0 + threadIdx.x, lrec + kCamRec * threadIdx.x);
    }
  } else {
  int skey[SH_SUB], srank[SH_SUB], spath[SH_SUB];
#pragma unroll
  for (int sub = 0; sub < SH_SUB; sub++) {
    const unsigned int j = (unsigned)sub * 256u + threadIdx.x;
    skey[sub] = 0; srank[sub] = 0; spath[sub] = 0;
    if (j < nblk) {
      spath[sub] = S.active[in][base + j];
      skey[sub] = shade_key(P, S, spath[sub]);
      srank[sub] = (int)atomicAdd(&lhist[skey[sub]], 1u);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned int acc = 0;
    for (int k = 0; k < SH_KEYS; k++) { lofs[k] = acc; acc += lhist[k]; }
  }
  __syncthreads();
#pragma unroll
  for (int sub = 0; sub < SH_SUB; sub++)
    if ((unsigned)sub * 256u + threadIdx.x < nblk) lsort[lofs[skey[sub]] + srank[sub]] = spath[sub];
  }
  __syncthreads();
  for (int sub = 0; sub < SH_SUB; sub++) {
    const unsigned int jj = (unsigned)sub * 256u + threadIdx.x;
    const bool live = jj < nblk;
    int path = live ? lsort[jj] : 0;
    // (an idle lane's pointer is out of range and never read: shade_path reads rec only for live
    // paths; clamping it cost the CAM kernel 12 B of scratch)
    const float4* rec = camrec ? lrec + kCamRec * ((unsigned)path / nfr - base / nfr) : nullptr;
    const ShadeOut so = shade_path<BSDF, FUSE, CAM>(W, E, path, live, CAM || W.cam_n != 0, !CAM && W.pass != 0, nsamples, rec);
    const bool qShadow = so.qShadow, qCont = so.qCont, keep = qShadow || qCont;
    // shadow rays from the front of the block's staging list, continuations from the back: the
    // block's queue run is [shadow rays][continuations], so a trace wave's claim is mostly one
    // kind
    const unsigned int qs = wave_lds_append(&lc[0], qShadow ? 1u : 0u);
    const unsigned int qc = wave_lds_append(&lc[4], qCont ? 1u : 0u);
    if (qShadow) lq[qs] = (path << 1) | 1;
    if (qCont) lq[2 * 256 * SH_SUB - 1 - qc] = path << 1;
    const unsigned int ai = wave_lds_append(&lc[1], keep ? 1u : 0u);
    if (keep) la[ai] = path;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (W.split_out) {  // shadow rays and continuations to their own queues
      lc[2] = lc[0] ? atomicAdd(&S.cnt[cqs(out)], lc[0]) : 0u;
      lc[5] = lc[4] ? atomicAdd(&S.cnt[cq(out)], lc[4]) : 0u;
    } else {
      lc[2] = (lc[0] + lc[4]) ? atomicAdd(&S.cnt[cq(out)], lc[0] + lc[4]) : 0u;
    }
    lc[3] = lc[1] ? atomicAdd(&S.cnt[ca(out)], lc[1]) : 0u;
  }
  __syncthreads();
  if (W.split_out) {
    for (unsigned int j = threadIdx.x; j < lc[0]; j += 256u) S.queue_s[out][lc[2] + j] = lq[j];
    for (unsigned int j = threadIdx.x; j < lc[4]; j += 256u) S.queue[out][lc[5] + j] = lq[2 * 256 * SH_SUB - 1 - j];
  } else {
    for (unsigned int j = threadIdx.x; j < lc[0] + lc[4]; j += 256u)
      S.queue[out][lc[2] + j] = j < lc[0] ? lq[j] : lq[2 * 256 * SH_SUB - 1 - (j - lc[0])];
  }
  for (unsigned int j = threadIdx.x; j < lc[1]; j += 256u) S.active[out][lc[3] + j] = la[j];
  __syncthreads();
  }
  // per-wave counter flush
  for (int off = 32; off > 0; off >>= 1) {
    nrays += __shfl_xor(nrays, off);
    nsamples += __shfl_xor(nsamples, off);
  }
  if ((threadIdx.x & 63) == 0 && (nrays | nsamples)) {
    // (the launch's last waves all flush at once: spread over the shard lines)
    unsigned long long* st = P.stats + stats_shard(blockIdx.x * 4u + (threadIdx.x >> 6));
    atomicAdd(&st[0], nrays);
    atomicAdd(&st[1], nsamples);
  }
}

// ---------------------------------------------------------------------------- finish
// Path-persistent finisher for small batches (one frame per render call: the reference's own
// usage, main.cpp:175-200).  Every wavefront pass waits for its slowest ray (150-250 traversal
// steps at ~1 us each, whatever the pass size), so the late passes of a single 1080p frame cost
// ~0.2 ms each while tracing only thousands of rays.  After pass F-1's shade, wf_finish gives each
// remaining path one lane, which traces the path's queued rays (shadow, then continuation: the
// dual-cursor steps of wf_trace, fetching triangle and node together, tl_step_prefetch) and runs
// the path's shade step (shade_path, as wf_shade), bounce after bounce until the path ends; a
// lane whose path ended takes the next one from the active list, and a wave runs shade steps in
// batches of RT_FINISH_SHADE_MIN ready lanes (or when no lane is tracing), so a lane does not wait
// for the wave's slowest ray of every bounce.  Same device functions in the same order per path:
// the image and the ray count are unchanged.  (A per-wave profile measured in round 2: the
// finisher is bound by latency at 2 waves/SIMD over ~80 paths per wave, not by single long rays.)
#ifndef RT_FINISH_SHADE_MIN  // lanes waiting for a shade step before the wave runs one
#define RT_FINISH_SHADE_MIN 16
#endif
#ifndef RT_FINISH_PRIO  // wave priority 3 / 2 / 1 / 0 above this many / half / a quarter / fewer lanes holding a
// path: the finisher is issue-bound while its waves share the SIMDs, and half of its wave time is
// waves with <= 16 paths left, so full waves (the long bounce chains of costly pixels) go first.
// C3 1080p single frames -3.5% (32: -3.2%; two levels at 16 / 8 / 32: -2.8 / -2.5 / -2.1%)
#define RT_FINISH_PRIO 16
#endif
#ifndef RT_FINISH_COOP  // a drained wave with at most this many paths left (<= 16) moves to four lanes per
// path (tl_coop_step; 0: off).  C3 1080p one-frame calls at 3 finisher waves/SIMD: 16 / 4 paths
// -5.7 / -4.1% (the shade batch at 16 lanes), 16 with the shade batch at 64 lanes -6.6%
// (profiles/r04_ab_single_coop_finisher_w3_C3.log)
#define RT_FINISH_COOP 16
#endif
#ifndef RT_FINISH_COOP_SHADE_MIN  // the same in coop mode, in lanes (four per path): a wave of <= 16 paths
// shades once all of them wait (or none traces)
#define RT_FINISH_COOP_SHADE_MIN 64
#endif
#ifndef RT_FINISH_WPE  // at least 2 waves/SIMD (no spills): 1080p single frames 3.64 (4) / 3.50 (3) / 3.47 ms (2);
// the compiler then kept the kernel at <= 168 VGPRs (3 waves); with the coop step it needs the
// bound to stay there (2 waves: coop +3.6% instead of -6.6%)
#define RT_FINISH_WPE 3
#endif
template <bool BSDF, bool WIDE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RT_FINISH_WPE)))
void wf_finish(const WFParams W) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const KParams& P = W.K;
  const WFState& S = W.S;
  const int in = W.pass & 1;
  const unsigned int na = S.cnt[ca(in)];
  const int lane = (int)(threadIdx.x & 63);
  // only as many waves as the list can feed take part (one lane per path)
  if ((blockIdx.x * (TL_LANES / 64) + (threadIdx.x >> 6)) * 64u >= na) return;
  TraceStack TS;
  TS.KL = P.lds_entries;
#ifdef RT_CHECK
  TS.cap = P.stack_cap;
#endif
  TS.lds0 = reinterpret_cast<int2*>(smem);
  TS.lds = TS.lds0 + threadIdx.x;
  TS.ovf = (gu64*)(P.stack_ovf) + blockIdx.x * TL_LANES;
  TS.ovs = P.ovf_lanes;
  const bool cull = (P.flags & RT_FLAG_NO_CULL) == 0;
  unsigned long long nrays = 0, nsamples = 0, nsteps = 0;
#ifdef RT_FINISH_PROF  // (make variant HIPEXTRA=-DRT_FINISH_PROF) RT_DEBUG_PASSES: per-wave {t0, t1, trace iterations | shade steps << 20 | paths << 40, shade time}
  const unsigned long long prof_t0 = wall_clock64();
  unsigned long long prof_it = 0, prof_sh = 0, prof_paths = 0, prof_sh_t = 0;
  unsigned long long prof_at[3] = {0, 0, 0}, prof_it_at[3] = {0, 0, 0};  // first time <= 16 / 4 / 1 lanes hold a path
#endif
  // lane state: no path / tracing the path's queued rays / rays done, waiting for its shade step
  enum : int { FS_IDLE = 0, FS_TRACE = 1, FS_SHADE = 2 };
  int st = FS_IDLE, path = 0;
  bool drained = false, contNext = false;
  int coop = 0;  // lanes per path: 0 (one) or 4 (RT_FINISH_COOP); wave-uniform
  auto lead = [&]() { return coop == 0 || (lane & (coop - 1)) == 0; };  // counts for its group
  TraceLane L;
  L.anyhit = false;
  L.sp = 0;  // (defined for lanes that never hold a path: the coop move reads every lane's)
  // first queued ray of the path: the shadow ray (any-hit) if any, then the continuation, whose
  // 24 B are fetched together with the shadow ray's and held until it starts (no load in the
  // trace loop)
  float4 ca = make_float4(0, 0, 0, 0);
  float2 cb = make_float2(0, 0);
  auto begin_rays = [&](bool sh, bool co) {
    contNext = sh && co;
    L.anyhit = sh;
    const float4 oa = sh ? S.sa[path] : S.ra[path];
    const float2 ob = sh ? S.sb[path] : S.rb[path];
    if (contNext) {
      ca = S.ra[path];
      cb = S.rb[path];
    }
    L.ox = oa.x; L.oy = oa.y; L.oz = oa.z;
    L.dx = oa.w; L.dy = ob.x; L.dz = ob.y;
    tl_start<WIDE>(P, L);
  };
  auto begin_cont = [&]() {
    contNext = false;
    L.anyhit = false;
    L.ox = ca.x; L.oy = ca.y; L.oz = ca.z;
    L.dx = ca.w; L.dy = cb.x; L.dz = cb.y;
    tl_start<WIDE>(P, L);
  };
  while (true) {
    // idle lanes take the next paths of the active list (one atomic per wave)
    const unsigned long long idle = __ballot(st == FS_IDLE);
    if (idle && !drained) {
      const unsigned int want = (unsigned int)__popcll(idle);
      unsigned int base = 0;
      if (lane == 0) base = atomicAdd(&S.cnt[kCntFetch], want);
      base = __builtin_amdgcn_readfirstlane(__shfl(base, 0));
      const unsigned int idx = base + (unsigned int)__popcll(idle & ((1ull << lane) - 1ull));
#ifdef RT_FINISH_PROF
      if (base < na) prof_paths += min(want, na - base);
#endif
      if (st == FS_IDLE && idx < na) {
        path = S.active[in][idx];
        const uint32_t flags = S.s5[path].y & 0xffu;
        st = FS_TRACE;  // a listed path always has a ray queued (wf_shade's keep)
        begin_rays((flags & PF_SHADOW) != 0, (flags & PF_CONT) != 0);
      }
      drained = base + want >= na;
    }
#if RT_FINISH_COOP
    if (WIDE && coop == 0 && drained) {
      // paths left: one per lane
      const unsigned long long live = __ballot(st != FS_IDLE);
      const int nl = __popcll(live);
      if (nl > 0 && nl <= RT_FINISH_COOP) {
        // the g-th path moves to lanes 4g .. 4g+3
        const int src = coop_move<4>(L, TS, live, lane, P.stack_cap);
        const int g = lane / 4;
        coop = 4;
        path = __shfl(path, src);
        contNext = __shfl((int)contNext, src) != 0;
        ca.x = __shfl(ca.x, src); ca.y = __shfl(ca.y, src); ca.z = __shfl(ca.z, src); ca.w = __shfl(ca.w, src);
        cb.x = __shfl(cb.x, src); cb.y = __shfl(cb.y, src);
        const int st_src = __shfl(st, src);  // (outside the select: a lane-permute from a lane masked off reads 0)
        st = g < nl ? st_src : (int)FS_IDLE;
      }
    }
#endif
    if (!__any(st != FS_IDLE)) break;
    {  // fuller waves issue first (s_setprio by the lanes holding a path; see RT_FINISH_PRIO)
      const int busy = __popcll(__ballot(st != FS_IDLE));
      if (busy > RT_FINISH_PRIO) __builtin_amdgcn_s_setprio(3);
      else if (busy > RT_FINISH_PRIO / 2) __builtin_amdgcn_s_setprio(2);
      else if (busy > RT_FINISH_PRIO / 4) __builtin_amdgcn_s_setprio(1);
      else __builtin_amdgcn_s_setprio(0);
    }
    // trace until enough lanes wait for their shade step (or none is tracing): a lane never waits
    // for the wave's slowest ray of every bounce, only for a batch of shade steps
    while (true) {
      const unsigned long long tr = __ballot(st == FS_TRACE);
      if (!tr || __popcll(__ballot(st == FS_SHADE)) >= (coop ? RT_FINISH_COOP_SHADE_MIN : RT_FINISH_SHADE_MIN)) break;
#ifdef RT_FINISH_PROF
      prof_it++;
      if (drained) {
        const int busy = __popcll(__ballot(st != FS_IDLE));
        const int lim[3] = {16, 4, 1};
        for (int q = 0; q < 3; q++)
          if (!prof_at[q] && busy <= lim[q]) { prof_at[q] = wall_clock64(); prof_it_at[q] = prof_it; }
      }
#endif
      if (st == FS_TRACE &&
          (!P.has_scene || (RT_FINISH_COOP && WIDE && coop == 4 ? tl_coop_step<4>(P, L, TS, cull, lane & 3)
                                                                : tl_step_prefetch<WIDE>(P, L, TS, cull)))) {
        S.res[2 * path + (L.anyhit ? 1 : 0)] = L.besttri;
        if (lead()) nrays++;
        if (contNext) begin_cont();
        else st = FS_SHADE;
      }
    }
    if (__any(st == FS_SHADE)) {
#ifdef RT_FINISH_PROF
      const unsigned long long ts = wall_clock64();
      prof_sh++;
#endif
      const bool sh = st == FS_SHADE;
      // the shade step reads its parameters through an opaque copy of the kernel-argument address,
      // so their ~30 pointers are loaded here (scalar loads) instead of being held in SGPRs
      // across the trace loop
      typedef const __attribute__((address_space(4))) WFParams KArgW;
      KArgW* Wk = (KArgW*)__builtin_amdgcn_kernarg_segment_ptr();  // W is the only argument
      asm volatile("" : "+s"(Wk));
      const WFParams* Wl = (const WFParams*)Wk;
      const KParams& PL = Wl->K;
      const Env EL{PL.hdr, PL.cache, PL.light, PL.hdr_w, PL.hdr_h, PL.hdr_res, PL.env_angle, PL.env_intensity};
      unsigned long long ns = 0;  // (a coop group runs its path's shade step on all its lanes: counted once)
      const ShadeOut o = shade_path<BSDF, true>(*Wl, EL, path, sh, false, true, ns);
      if (lead()) nsamples += ns;
      if (sh) {
        if (lead()) nsteps++;
        if (o.qShadow || o.qCont) {
          st = FS_TRACE;
          begin_rays(o.qShadow, o.qCont);
        } else {
          st = FS_IDLE;
        }
      }
#ifdef RT_FINISH_PROF
      prof_sh_t += wall_clock64() - ts;
#endif
    }
  }
#ifdef RT_FINISH_PROF
  if (P.wave_log && lane == 0) {
    unsigned long long* w = P.wave_log + 8 * ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6));
    w[0] = prof_t0; w[1] = wall_clock64(); w[2] = prof_it | (prof_sh << 20) | (prof_paths << 40); w[3] = prof_sh_t;
    for (int q = 0; q < 3; q++) w[4 + q] = prof_at[q] ? ((prof_at[q] - prof_t0) | (prof_it_at[q] << 32)) : 0ull;
  }
#endif
  for (int off = 32; off > 0; off >>= 1) {
    nrays += __shfl_xor(nrays, off);
    nsamples += __shfl_xor(nsamples, off);
    nsteps += __shfl_xor(nsteps, off);
  }
  if (lane == 0) {
    unsigned long long* st = P.stats + stats_shard(blockIdx.x * 4u + (threadIdx.x >> 6));
    atomicAdd(&st[0], nrays);
    atomicAdd(&st[1], nsamples);
    atomicAdd(&st[2], nsteps);  // rt_stats.finish_steps
  }
}

}  // namespace rtd
