/* rt_abi.h — C-ABI of the MI355X path tracer (librtamd.so, HIP for gfx950).
 *
 * Drop-in replacement for the reference's OpenGL program interface of the path-tracing
 * fragment shader (src/shaders/fragment_shader_ray_tracing.glsl, "RT:"), which the
 * reference drives from src/sources/main.cpp.  Entry point -> reference interface:
 *
 *   rt_create / rt_destroy   <- Shader RayTracerShader(...) + GL context (src/core/Shader.h:21-108,
 *                               main.cpp:93-95)
 *   rt_set_scene             <- EncodedBVHandTriangles() glBufferData/glTexBuffer uploads of the
 *                               triangle and BVH texture buffers (src/core/Scene.h:240-256) and the
 *                               nTriangles/nNodes uniforms (main.cpp:135-136); SoA instead of AoS
 *   rt_set_scene_encoded     <- the same upload taking the reference's AoS encodings verbatim
 *                               (Triangle_encoded src/core/Triangle.h:28-39, BVHNode_encoded
 *                               src/core/BVH.h:17-21)
 *   rt_update_materials      <- RefreshTriangleMaterial re-upload (src/core/Triangle.h:133-151),
 *                               with post-BVH triangle indices
 *   rt_set_env               <- InitHdrEnvMap() hdrMap/hdrCache RGB32F textures + hdrResolution
 *                               (src/core/Scene.h:164-184, main.cpp:138, :149-155)
 *   rt_resize                <- RenderBuffer::Init/Resize RGB32F ping-pong FBOs (src/core/Screen.h:110-122)
 *                               + this rank's pixel tiles (multi-GPU sharding, new)
 *   rt_reset / rt_set_loop_num <- camera.LoopNum = 0 (main.cpp:326, src/core/Camera.h:453)
 *   rt_render(_async)        <- per-frame loop body main.cpp:175-200: LoopIncrease, setCurrentBuffer,
 *                               the uniform list of main.cpp:181-199, DrawScreen
 *   rt_read_accum            <- reading the accumulation texture (Utility.h:19-30 SaveFrame reads it
 *                               after tone mapping; here the raw fp32 history)
 *   rt_accum_device / rt_assemble_frame <- (new) device-side tile gather for RCCL
 *
 * Conventions: every function returns RT_OK (0) or a negative rt_err_*; nothing aborts.
 * A context is bound to one HIP device and is not thread-safe (one host thread per ctx),
 * matching the single GL context of the reference (main.cpp:72).
 */
#ifndef RT_ABI_H
#define RT_ABI_H

#include <stddef.h>
#include <stdint.h>

/* ABI version of this header.
 * 4: rt_stats gained pass0_steps, pass1_steps, finish_steps and trace_busy_ms (round 4; round 3
 *    had added path_steps and p1_rays), and rt_stats_get_sized / rt_abi_version / RT_FLAG_SERIAL
 *    appeared.  path_steps changed meaning in 4: it counts wf_shade steps only; the finisher's shade
 *    steps, which it included before, are finish_steps (their sum is the old path_steps).
 * 5: rt_stats_get and rt_render write the ABI-3 struct only (the 104 bytes through p1_rays, what
 *    every binding of an ABI-3 header allocated; ABI 4 wrote past them), and the fields added in 4
 *    reach a caller only through rt_stats_get_sized with its own sizeof(rt_stats).  A binding
 *    written against the ABI-4 header (whose rt_stats_get filled the whole struct) must switch to
 *    rt_stats_get_sized(ctx, &s, sizeof s) to keep pass0_steps .. trace_busy_ms: the layout is
 *    unchanged, so that call with the ABI-4 size fills them (tests/c/abi_stats.c).
 *    RT_FLAG_SORTED_TRAVERSAL is accepted and has no effect (the octant-ordered traversal it
 *    switched off was removed).
 * 6: rt_gather moves the tiles with RCCL when the contexts sit on distinct devices;
 *    rt_gather_ex chooses the transport, rt_gather_last_transport reports it.  Nothing else changed.
 * A binding checks rt_abi_version() at load time. */
#define RT_ABI_VERSION 6

#ifdef __cplusplus
extern "C" {
#endif

enum {
  RT_OK = 0,
  RT_ERR_ARG = -1,
  RT_ERR_HIP = -2,      /* a HIP runtime call failed; rt_last_error() has the text */
  RT_ERR_STATE = -3,    /* call order (e.g. render before set_scene/resize)          */
  RT_ERR_NOMEM = -4,
  RT_ERR_NODEVICE = -5, /* no HIP device / bad ordinal                               */
  RT_ERR_LIMIT = -6     /* scene exceeds a kernel limit (leaf > 16 tris, depth > 64) */
};

/* Frames per kernel batch; the path-state budget (184 B per pixel-frame; rt_set_max_paths or
 * RT_MAX_SLOTS, default 320 Mi slots = 64 GB) bounds it too: 161 frames at 1920x1080 with the
 * default budget; bench.py raises the budget to a whole 1024-frame step, which one GPU runs as two
 * launches of 512 frames (206 GB) and each of 8 tile-sharded GPUs as one launch (51 GB). */
enum { RT_MAX_FRAMES_PER_LAUNCH = 1024 };

/* Disney material (src/core/Material.h:25-46), 24 floats, same layout as rts_material. */
typedef struct rt_material {
  float emissive[3];
  float base_color[3];
  float subsurface, metallic, specular, specular_tint, roughness, anisotropic;
  float sheen, sheen_tint, clearcoat, clearcoat_gloss, ior, transmission;
  float medium_color[3];
  float medium_type, medium_density, medium_anisotropy;
} rt_material;

/* Scene in post-BVH triangle order (what buildBVHwithSAH leaves in `triangles`). */
typedef struct rt_scene_soa {
  int32_t n_triangles;
  const float *p1, *p2, *p3;      /* float[3*n_triangles], xyz interleaved */
  const float *n1, *n2, *n3;      /* vertex normals, float[3*n_triangles]  */
  const int32_t* material_id;     /* [n_triangles] index into materials    */
  const rt_material* materials;
  int32_t n_materials;
  int32_t n_nodes;                /* reference numbering: node 0 dummy, root 1, child 0 = none */
  const int32_t *node_left, *node_right, *node_n, *node_index;
  const float *node_aa, *node_bb; /* float[3*n_nodes] */
} rt_scene_soa;

/* Pixel tiling: the frame is cut into tile_w x tile_h tiles (multiples of 8), numbered
 * row-major from the bottom-left; this context renders tiles t with t % world == rank. */
typedef struct rt_tiling {
  int32_t tile_w, tile_h, rank, world;
} rt_tiling;

/* Per-call uniforms (main.cpp:181-199).  screen size comes from rt_resize. */
typedef struct rt_frame_params {
  float position[3], front[3], right[3], up[3], left_bottom_corner[3];
  float half_h, half_w;
  int32_t enable_mis, enable_env_map, enable_bsdf;
  float env_intensity, env_angle;
  int32_t max_bounce, max_iterations;
  int32_t flags;                  /* RT_FLAG_* */
} rt_frame_params;

enum {
  RT_FLAG_NO_CULL = 1,            /* disable closest-hit box culling (exhaustive RT:338 order)  */
  RT_FLAG_COUNT_VISITS = 2,       /* also count node/triangle visits (slower)                  */
  RT_FLAG_MEGAKERNEL = 4,         /* single persistent megakernel instead of the wavefront path */
  RT_FLAG_NO_FINISH = 8,          /* never end paths in the path-persistent finisher            */
  RT_FLAG_FINISH = 16,            /* use the finisher whatever the batch size (rt_set_finish)   */
  RT_FLAG_SERIAL = 32,            /* measurement: one frame group per batch (no two groups' kernels
                                     overlap), at most one group's path state of frames per batch */
  RT_FLAG_SORTED_TRAVERSAL = 64   /* ABI 4 (accepted, no effect since ABI 5): the trace always visits
                                     children by entry distance */
};

typedef struct rt_stats {
  uint64_t rays;            /* hitBVH invocations: camera + NEE shadow + continuation    */
  uint64_t samples;         /* pixel samples traced (frames x pixels, R12 copies excluded) */
  uint64_t internal_pops, leaf_pops, tri_tests;  /* only with RT_FLAG_COUNT_VISITS */
  uint64_t launches;        /* rt_render_async calls that launched work                  */
  double kernel_ms;         /* GPU time of those calls (HIP events on the ctx stream)     */
  uint64_t trace_launches;  /* traversal kernel launches (wavefront) / megakernel launches */
  double trace_ms;          /* summed duration of those launches (HIP events around each) */
  uint64_t trace_iters;     /* RT_FLAG_COUNT_VISITS: traversal loop iterations, all waves */
  uint64_t trace_iters_max; /* RT_FLAG_COUNT_VISITS: max loop iterations of one wave       */
  uint64_t path_steps;      /* wavefront path: wf_shade steps (one per path per bounce pass; since
                               ABI 4 without the finisher's, which are finish_steps)           */
  uint64_t p1_rays;         /* wavefront path: rays traced from pass 0's 16-B ray records  */
  /* ---- ABI 4: written only by rt_stats_get_sized */
  uint64_t pass0_steps;     /* of path_steps: pass 0 (implicit camera paths)                */
  uint64_t pass1_steps;     /* of path_steps: pass 1 (paths whose rays are 16-B records)    */
  uint64_t finish_steps;    /* shade steps run by the path-persistent finisher (wf_finish)  */
  double trace_busy_ms;     /* union of the traversal launches' intervals: the time during
                               which at least one of them ran (frame groups overlap, so
                               trace_ms can exceed it)                                       */
} rt_stats;

typedef struct rt_ctx rt_ctx;

int rt_create(int hip_device, rt_ctx** out);
int rt_destroy(rt_ctx* ctx);
const char* rt_last_error(const rt_ctx* ctx);
/* Device properties used for the launch geometry (CUs, clock). */
int rt_device_info(const rt_ctx* ctx, int32_t* n_cus, int32_t* blocks_per_cu, int32_t* lds_bytes_per_block);

int rt_set_scene(rt_ctx* ctx, const rt_scene_soa* scene);
int rt_set_scene_encoded(rt_ctx* ctx, const float* tri_enc, int32_t n_triangles, const float* node_enc,
                         int32_t n_nodes);
int rt_update_materials(rt_ctx* ctx, int32_t first, int32_t count, const rt_material* material);
/* hdr_rgb / cache_rgb: w*h*3 floats, row 0 = first uploaded row (texture v = 0). */
int rt_set_env(rt_ctx* ctx, const float* hdr_rgb, const float* cache_rgb, int32_t w, int32_t h,
               int32_t hdr_resolution);
int rt_resize(rt_ctx* ctx, int32_t width, int32_t height, const rt_tiling* tiling /* NULL = whole frame */);
int rt_reset(rt_ctx* ctx);                       /* LoopNum = 0 (history kept, as the FBOs are) */
int rt_set_loop_num(rt_ctx* ctx, int32_t loop_num);
int rt_get_loop_num(const rt_ctx* ctx, int32_t* loop_num);
/* Clear this rank's accumulation to zero (fresh FBO contents). */
int rt_clear_accum(rt_ctx* ctx);
/* Tile ownership (SURVEY §8(e) "by a cost estimate from frame 1"): owner[t] = the rank that renders
 * global tile t (row-major from the bottom-left, n_tiles = tiles_x * tiles_y of the rt_resize
 * tiling).  rt_resize sets owner[t] = t % world; every rank of a job must set the same map.  Local
 * order = ascending tile id.  Re-sizes the accumulation (zeroed) and the pixel list, resets LoopNum. */
int rt_set_tile_owners(rt_ctx* ctx, const int32_t* owner, int32_t n_tiles);
int rt_get_tile_owners(const rt_ctx* ctx, int32_t* owner, int32_t n_tiles);
/* Cost probe for rt_set_tile_owners: renders n_frames and returns, per LOCAL tile of this ctx,
 * its rays' BVH node + triangle steps plus a per-ray share (deterministic integers).  LoopNum and
 * the accumulation are left as they were; the stats counters include the probe frames. */
int rt_tile_costs(rt_ctx* ctx, const rt_frame_params* params, const float* rand_origin, int32_t n_frames,
                  uint64_t* costs);
/* Longest-first work order (no GL counterpart: the rasteriser schedules fragments itself).  Traces
 * the camera pass of n_frames as a cost probe (the camera rays are the same in every frame, so the
 * costs do not depend on the frames; state left unchanged), then reorders this ctx's pixel
 * list by whole 64-pixel blocks (an 8x8 block stays one wave) in descending cost, so the blocks
 * whose rays cost most are queued first and a pass's tail is the cheap blocks; the costliest 5%
 * become a pixel group of their own in one-frame calls (their long bounce chains reach the
 * path-persistent finisher early, beside the rest's first passes).  Results are
 * unchanged (pixels are independent; the accumulation keeps its layout); rt_resize and
 * rt_set_tile_owners restore the natural order. */
int rt_order_work(rt_ctx* ctx, const rt_frame_params* params, const float* rand_origin, int32_t n_frames);
/* Path-state budget in pixel-frames (184 B each): frames in flight per launch = slots / pixels of
 * this rank, at most RT_MAX_FRAMES_PER_LAUNCH.  0 = RT_MAX_SLOTS from the environment or the
 * default 320 Mi slots.  A budget beyond free device memory runs fewer frames at a time.  No GL
 * counterpart: the fragment shader has one path per pixel in flight. */
int rt_set_max_paths(rt_ctx* ctx, uint64_t slots);
/* Path-persistent finisher (no GL counterpart: main.cpp:175-200 draws one frame per loop pass,
 * and each wavefront pass of such a small batch waits for its slowest ray).  A frame group of at
 * most max_slots path slots runs passes 0 .. pass-1 as wavefront passes and then ends every path
 * in one launch, one lane per path (results unchanged).  pass 0 disables it; defaults 2 and 8 Mi
 * slots (1080p: up to 8 frames per group).  RT_FLAG_NO_FINISH / RT_FLAG_FINISH override per call. */
int rt_set_finish(rt_ctx* ctx, int32_t pass, uint64_t max_slots);
/* Frames in flight across one-frame calls (the GL driver's own frame queue: main.cpp:175-251
 * issues a draw per loop pass and glfwSwapBuffers does not wait for it to finish).  With depth
 * 2 (the most; 1 = off), a one-frame rt_render_async call made while the previous call is
 * still running runs on the other of two internal streams with its own path state, so call k+1's
 * early passes overlap call k's latency-bound last bounces (a call with nothing in flight keeps
 * the lower-latency split into pixel groups).  Calls of one batch are pipelined the same way when
 * two sets of their path state fit the budget.  Only call k+1's blend waits for the ctx stream (call k's blend and
 * whatever the caller queued there since), and the ctx stream still joins every call at its end:
 * results and ordering are those of depth 1.  Default 1; synchronises the ctx. */
int rt_set_pipeline(rt_ctx* ctx, int32_t depth);

/* Enqueue n_frames progressive frames (one randOrigin per frame) on the ctx stream.  Each
 * frame first applies main.cpp:175 (LoopNum++ unless it reached max_iterations). */
int rt_render_async(rt_ctx* ctx, const rt_frame_params* params, const float* rand_origin, int32_t n_frames);
/* rt_render_async + synchronise + optional stats snapshot. */
int rt_render(rt_ctx* ctx, const rt_frame_params* params, const float* rand_origin, int32_t n_frames,
              rt_stats* stats /* ABI-3 fields only (see rt_stats_get) */);
int rt_synchronize(rt_ctx* ctx);
int rt_stats_get(rt_ctx* ctx, rt_stats* stats);  /* synchronises; writes the ABI-3 fields (104 bytes) */
/* The same, writing at most stats_bytes bytes (a caller's own, possibly older, sizeof(rt_stats)). */
int rt_stats_get_sized(rt_ctx* ctx, rt_stats* stats, size_t stats_bytes);
int rt_stats_reset(rt_ctx* ctx);
int rt_abi_version(void);                        /* RT_ABI_VERSION the library was built with */

/* The HIP stream (hipStream_t) the ctx launches on, for external events / collectives. */
int rt_get_stream(const rt_ctx* ctx, void** stream);
int rt_set_stream(rt_ctx* ctx, void* stream /* NULL = ctx-owned stream */);

enum { RT_LAYOUT_FRAME = 0, RT_LAYOUT_LOCAL_TILES = 1 };
/* FRAME: rgb_out = width*height*3 floats, row 0 = bottom row (GL framebuffer order); only this
 * rank's pixels are written.  LOCAL_TILES: local_tiles*tile_h*tile_w*3 floats. */
int rt_read_accum(rt_ctx* ctx, float* rgb_out, int32_t layout);
/* Upload a history (same layouts) — e.g. resume from a saved accumulation. */
int rt_write_accum(rt_ctx* ctx, const float* rgb_in, int32_t layout);
/* Device accumulation buffer: float4 (rgb + pad) per local tile pixel, padded to
 * max_local_tiles tiles so that every rank's buffer has the same size. */
int rt_accum_device(const rt_ctx* ctx, void** device_ptr, size_t* bytes, int32_t* local_tiles,
                    int32_t* max_local_tiles);
/* Device-to-device copy of the accumulation buffer (rt_accum_device bytes) into dst, enqueued
 * on the ctx stream (feeds the frame-end gather). */
int rt_copy_accum_device(rt_ctx* ctx, void* dst_device, size_t bytes);
/* Un-permute `world` gathered accumulation buffers (rank-major, each rt_accum_device bytes) on
 * this ctx's device into a width*height*3 float frame (device pointer). */
int rt_assemble_frame(rt_ctx* ctx, const void* gathered_device, int32_t world, void* frame_device);
/* Single-process form of the frame-end gather (SURVEY §8(b) rt_gather, §8(e)): ctxs[r] renders
 * rank r of a world of n (rt_resize tiling; one context per device, or several on one).  After
 * the work queued on each context, its accumulation tiles reach ctxs[0]'s device, are un-permuted
 * there (rt_assemble_frame) and read back: full_rgb = width*height*3 floats, row 0 = bottom
 * (RT_LAYOUT_FRAME).  Transport: with one device per context an RCCL gather over xGMI
 * (ncclCommInitAll over the contexts' devices, kept in ctxs[0]; ncclSend from every rank's stream,
 * ncclRecv on rank 0's, in one group), else peer copies (several contexts on one device).
 * Synchronous; errors land in rt_last_error(ctxs[0]).  One process per GPU uses
 * rt_copy_accum_device + a torch.distributed (RCCL) gather + rt_assemble_frame instead (bench.py). */
int rt_gather(rt_ctx* const* ctxs, int32_t n, float* full_rgb);
enum { RT_GATHER_AUTO = 0, RT_GATHER_RCCL = 1, RT_GATHER_PEER = 2 };
/* rt_gather with the transport chosen: RT_GATHER_AUTO (rt_gather's rule), RT_GATHER_RCCL
 * (RT_ERR_ARG unless every context has its own device), RT_GATHER_PEER (hipMemcpyPeerAsync). */
int rt_gather_ex(rt_ctx* const* ctxs, int32_t n, float* full_rgb, int32_t transport);
/* The transport ctx's last rt_gather / rt_gather_ex as ctxs[0] used (RT_GATHER_RCCL or
 * RT_GATHER_PEER; 0 before any). */
int rt_gather_last_transport(const rt_ctx* ctx);

/* Display / screenshot — replaces the tone-mapping pass
 * (src/shaders/fragment_shader_tone_mapping.glsl:66-93, main.cpp:215-227) or the screen blit
 * (fragment_shader_screen.glsl:6-9) plus the 8-bit read-back of SaveFrame (Utility.h:19-30).
 * flags: RT_DISPLAY_TONEMAP (enableToneMapping: simpleACES), RT_DISPLAY_GAMMA
 * (enableGammaCorrection: pow(c, 1/2.2), only with TONEMAP, as in main.cpp:216).
 * frame_device: an assembled width*height*3 float frame (rt_assemble_frame), or NULL for this
 * context's own accumulation (single rank only).  rgb8_host: width*height*3 bytes, row 0 = top
 * (PNG order).  Synchronous. */
enum { RT_DISPLAY_TONEMAP = 1, RT_DISPLAY_GAMMA = 2 };
int rt_tonemap(rt_ctx* ctx, const float* frame_device, int32_t flags, uint8_t* rgb8_host);
/* The same display pass without waiting for it (main.cpp:228-251: the blit and glfwSwapBuffers
 * queue the frame and the loop goes on): enqueues the pass and its read-back into internal pinned
 * slot `slot` (0..3) on the ctx stream, after the render calls queued before it, and returns.  A
 * render call queued afterwards blends only after this pass has read the accumulation.
 * rt_display_fetch waits for that slot's image and copies it out (width*height*3 bytes). */
int rt_tonemap_async(rt_ctx* ctx, const float* frame_device, int32_t flags, int32_t slot);
int rt_display_fetch(rt_ctx* ctx, int32_t slot, uint8_t* rgb8_host);

#ifdef __cplusplus
}
#endif
#endif
