/* A C binding of include/rt_abi.h: what a caller compiled against the header sees of
 * rt_stats.  Renders two frames of a one-triangle scene, then checks that
 *   - rt_stats_get writes the ABI-3 prefix only (104 bytes; bytes past it keep the caller's fill),
 *   - rt_stats_get_sized with the ABI-4 size (this header's sizeof(rt_stats): ABI 5 kept the ABI-4
 *     layout) reaches the ABI-4 tail: pass0_steps and trace_busy_ms are set.
 * Exit status 0 on success; built by __graft_entry__.build() (gcc, links lib/librtamd.so), run by
 * tests/test_abi.py on the GPU box. */
#include <stddef.h>
#include <stdio.h>
#include <string.h>

#include "rt_abi.h"

#define CHECK(x)                                                                 \
  do {                                                                           \
    int rc_ = (x);                                                               \
    if (rc_ != RT_OK) {                                                          \
      fprintf(stderr, "%s failed: %d (%s)\n", #x, rc_, ctx ? rt_last_error(ctx) : ""); \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

int main(void) {
  rt_ctx* ctx = NULL;
  if (rt_abi_version() != RT_ABI_VERSION) {
    fprintf(stderr, "library ABI %d, header %d\n", rt_abi_version(), RT_ABI_VERSION);
    return 1;
  }
  CHECK(rt_create(0, &ctx));
  const float p1[3] = {-1.0f, -1.0f, 0.0f}, p2[3] = {1.0f, -1.0f, 0.0f}, p3[3] = {0.0f, 1.0f, 0.0f};
  const float n[3] = {0.0f, 0.0f, 1.0f};
  const int32_t mid = 0;
  rt_material m;
  memset(&m, 0, sizeof m);
  m.base_color[0] = m.base_color[1] = m.base_color[2] = 0.5f;
  m.roughness = 0.5f;
  m.ior = 1.5f;
  m.medium_color[0] = m.medium_color[1] = m.medium_color[2] = 1.0f;
  /* node 0 dummy, node 1 = the root, a leaf holding triangle 0 */
  const int32_t left[2] = {0, 0}, right[2] = {0, 0}, nn[2] = {0, 1}, idx[2] = {0, 0};
  const float aa[6] = {0, 0, 0, -1.0f, -1.0f, 0.0f}, bb[6] = {0, 0, 0, 1.0f, 1.0f, 0.0f};
  rt_scene_soa s = {1, p1, p2, p3, n, n, n, &mid, &m, 1, 2, left, right, nn, idx, aa, bb};
  CHECK(rt_set_scene(ctx, &s));
  const float env[6] = {1.0f, 1.0f, 1.0f, 1.0f, 1.0f, 1.0f};
  CHECK(rt_set_env(ctx, env, env, 2, 1, 2));
  CHECK(rt_resize(ctx, 16, 16, NULL));
  rt_frame_params fp;
  memset(&fp, 0, sizeof fp);
  const float pos[3] = {0.0f, 0.0f, 3.0f}, front[3] = {0.0f, 0.0f, -1.0f}, rgt[3] = {1.0f, 0.0f, 0.0f},
              up[3] = {0.0f, 1.0f, 0.0f}, lbc[3] = {-0.5f, -0.5f, -1.0f};
  memcpy(fp.position, pos, sizeof pos);
  memcpy(fp.front, front, sizeof front);
  memcpy(fp.right, rgt, sizeof rgt);
  memcpy(fp.up, up, sizeof up);
  memcpy(fp.left_bottom_corner, lbc, sizeof lbc);
  fp.half_h = fp.half_w = 0.5f;
  fp.enable_mis = fp.enable_env_map = fp.enable_bsdf = 1;
  fp.env_intensity = 1.0f;
  fp.max_bounce = 2;
  fp.max_iterations = -1;
  const float ro[2] = {674764.0f, 1000000.0f};
  CHECK(rt_render(ctx, &fp, ro, 2, NULL));

  unsigned char buf[sizeof(rt_stats) + 64];
  memset(buf, 0xAB, sizeof buf);
  CHECK(rt_stats_get(ctx, (rt_stats*)buf));
  const size_t abi3 = offsetof(rt_stats, pass0_steps);
  for (size_t i = abi3; i < sizeof buf; i++)
    if (buf[i] != 0xAB) {
      fprintf(stderr, "rt_stats_get wrote byte %zu past the ABI-3 prefix (%zu bytes)\n", i, abi3);
      return 1;
    }
  rt_stats st;
  memset(&st, 0, sizeof st);
  CHECK(rt_stats_get_sized(ctx, &st, sizeof st));
  if (st.rays == 0 || st.samples != 2 * 16 * 16 || st.pass0_steps == 0 || !(st.trace_busy_ms > 0.0)) {
    fprintf(stderr, "ABI-4 tail not reached: rays %llu samples %llu pass0_steps %llu trace_busy_ms %g\n",
            (unsigned long long)st.rays, (unsigned long long)st.samples, (unsigned long long)st.pass0_steps,
            st.trace_busy_ms);
    return 1;
  }
  printf("abi_stats ok: rays %llu, pass0_steps %llu, trace_busy_ms %.4f\n", (unsigned long long)st.rays,
         (unsigned long long)st.pass0_steps, st.trace_busy_ms);
  CHECK(rt_destroy(ctx));
  return 0;
}
