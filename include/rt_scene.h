/* rt_scene.h — host-side scene preparation C-ABI (CPU, C++17 implementation in
 * opengl-ray-tracing-framework_amd/csrc/host/rt_scene.cpp, built as librtscene.so).
 *
 * Replaces the reference's host pipeline that feeds the path-tracing shader:
 *   rts_obj_load / rts_mesh_*      <- Model::loadModel/processNode/processMesh
 *                                     (src/core/Model.h:48-159; assimp flags :51-52)
 *   rts_scene_add_mesh             <- getTriangle + getTransformMatrix
 *                                     (src/core/Triangle.h:41-131, src/core/Model.h:250-266)
 *   rts_scene_build_bvh            <- buildBVHwithSAH with the dummy node 0
 *                                     (src/core/BVH.h:110-241, src/core/Scene.h:186-201)
 *   rts_scene_encode               <- EncodedBVHandTriangles / EncodeTriangle
 *                                     (src/core/Scene.h:203-238, src/core/Triangle.h:153-175)
 *   rts_scene_export_soa           <- (new) SoA hand-off to the HIP path (rt_abi.h)
 *   rts_scene_set_material         <- RefreshTriangleMaterial (src/core/Triangle.h:133-151),
 *                                     fixed to take post-BVH ranges
 *   rts_hdr_load                   <- HDRLoader::load (thirdparty/hdrloader/hdrloader.cpp:29-190),
 *                                     with the %ld-into-int bug fixed
 *   rts_hdr_cache                  <- calculateHdrCache (src/core/Utility.h:33-131)
 *   rts_camera                     <- Camera::updateCameraVectors (src/core/Camera.h:160-174)
 *   rts_cpu_rand_origins           <- main.cpp:190 randOrigin = 674764*(GetCPURandom()+1)
 *
 * Conventions: return 0 on success, negative rts_err_* on failure; never abort.
 * All arrays are caller-owned; counts are int32.
 */
#ifndef RT_SCENE_H
#define RT_SCENE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  RTS_OK = 0,
  RTS_ERR_ARG = -1,
  RTS_ERR_IO = -2,
  RTS_ERR_FORMAT = -3,
  RTS_ERR_STATE = -4,
  RTS_ERR_NOMEM = -5
};

/* Disney material, field-for-field src/core/Material.h:25-46 (texture ids dropped: the
 * path tracer never samples textures). */
typedef struct rts_material {
  float emissive[3];
  float base_color[3];
  float subsurface, metallic, specular, specular_tint, roughness, anisotropic;
  float sheen, sheen_tint, clearcoat, clearcoat_gloss, ior, transmission;
  float medium_color[3];
  float medium_type, medium_density, medium_anisotropy;
} rts_material;

typedef struct rts_mesh rts_mesh;     /* a post-processed (assimp-equivalent) model   */
typedef struct rts_scene rts_scene;   /* triangle list + BVH, src/core/RenderSettings.h:502 */

/* ---- meshes ------------------------------------------------------------------- */
/* parse_mode: 0 = correctly rounded strtof (default; reproduces the node counts measured from the
 * reference BVH.h in SURVEY.md §8(c)), 1 = restatement of assimp's fast_atoreal_move (assimp is
 * an unpinned, absent submodule: its last-ulp rounding differs on some coordinates). */
int rts_obj_load(const char* path, int parse_mode, rts_mesh** out);
/* Build from raw OBJ data (positions, optional file normals, polygon faces). */
int rts_mesh_from_raw(const float* positions, int n_positions, const float* normals, int n_normals,
                      const int32_t* face_sizes, int n_faces, const int32_t* pos_index,
                      const int32_t* nrm_index /* may be NULL */, rts_mesh** out);
/* Raw OBJ data as parsed (for the compact asset format), sizes first with NULL arrays. */
int rts_obj_parse_raw(const char* path, int parse_mode, int32_t* n_positions, int32_t* n_normals,
                      int32_t* n_faces, int32_t* n_indices, float* positions, float* normals,
                      int32_t* face_sizes, int32_t* pos_index, int32_t* nrm_index);
int rts_mesh_counts(const rts_mesh* m, int32_t* n_vertices, int32_t* n_indices);
/* Corner vertices (positions, normals) and triangle indices after post-processing. */
int rts_mesh_data(const rts_mesh* m, float* positions, float* normals, int32_t* indices);
void rts_mesh_free(rts_mesh* m);

/* ---- scene -------------------------------------------------------------------- */
int rts_scene_create(rts_scene** out);
void rts_scene_free(rts_scene* s);
/* getTriangle(meshes, triangles, material, getTransformMatrix(rotate, translate, scale), smooth).
 * Returns the [first, end) triangle range in *pre-BVH* order via range[2]. */
int rts_scene_add_mesh(rts_scene* s, const rts_mesh* m, const rts_material* mat, const float rotate_deg[3],
                       const float translate[3], const float scale[3], int smooth_normal, int32_t range[2]);
/* Append raw triangles (positions float[9*n]: p1,p2,p3 per triangle) with flat normals
 * normalize(cross(p2-p1, p3-p1)) and no normalisation/transform (probe and procedural use). */
int rts_scene_add_triangles(rts_scene* s, const float* positions, int n, const rts_material* mat, int32_t range[2]);
/* buildBVHwithSAH(triangles, nodes, 0, n-1, leaf_size) after the dummy node 0.
 * Reorders the scene's triangles in place (as the reference does). */
int rts_scene_build_bvh(rts_scene* s, int leaf_size);
int rts_scene_counts(const rts_scene* s, int32_t* n_triangles, int32_t* n_nodes, int32_t* max_depth,
                     int32_t* n_leaves);
/* Reference GPU encodings: tri_enc = n_tri*14*3 floats, node_enc = n_nodes*4*3 floats. */
int rts_scene_encode(const rts_scene* s, float* tri_enc, float* node_enc);
/* Raw node arrays (int left,right,n,index; float AA[3],BB[3]) in reference numbering. */
int rts_scene_nodes(const rts_scene* s, int32_t* left, int32_t* right, int32_t* n, int32_t* index, float* aa,
                    float* bb);
/* SoA hand-off in post-BVH order: positions p1|p2|p3 and normals n1|n2|n3 as float[3*n] each,
 * material id per triangle, and the de-duplicated material table (n_materials returned;
 * pass materials=NULL to query). */
int rts_scene_export_soa(const rts_scene* s, float* p1, float* p2, float* p3, float* n1, float* n2, float* n3,
                         int32_t* material_id, rts_material* materials, int32_t* n_materials);
/* Replace the material of post-BVH triangles [first, first+count). */
int rts_scene_set_material(rts_scene* s, int first, int count, const rts_material* mat);
/* Index (post-BVH) of the triangles that came from pre-BVH range [first, end). */
int rts_scene_post_bvh_index(const rts_scene* s, int32_t* pre_to_post);

/* ---- environment -------------------------------------------------------------- */
/* Radiance .hdr -> float RGB, rows in file order (top row first). *out_rgb allocated with
 * malloc; release with rts_free. */
int rts_hdr_load(const char* path, int32_t* width, int32_t* height, float** out_rgb);
/* hdrCache texels (x_sample/W, y_sample/H, pdf) for an RGB float image. */
int rts_hdr_cache(const float* rgb, int width, int height, float* out_cache);
void rts_free(void* p);

/* ---- camera / frame parameters ------------------------------------------------ */
/* out[17] = front[3], right[3], up[3], left_bottom_corner[3], half_h, half_w, (3 reserved) */
int rts_camera(float yaw_deg, float pitch_deg, float zoom_deg, float screen_ratio, float* out);
/* randOrigin_k = 674764 * (rand()/(RAND_MAX+1.0) + 1) after srand(seed) (main.cpp:190,
 * src/core/Utility.h:11-17), any n: glibc's rand() is restated in-tree (rts_glibc_rand), so the
 * list does not depend on the host libc. */
int rts_cpu_rand_origins(unsigned int seed, int n, float* out);
/* The first n values of glibc rand() after srand(seed) (stdlib/random_r.c TYPE_3 generator,
 * restated; identical to the libc's on glibc systems). */
int rts_glibc_rand(unsigned int seed, int n, int* out);

/* The HIP path's traversal records and edge-filter margin (csrc/common/tri_filter.h; rt_set_scene
 * builds them the same way): tri = 3 float[4] per triangle {p1, N.x} {p2, N.y} {p3, N.z}, out = 3
 * float[4] per triangle {p1, N.x} {R2, N.y} {R3, N.z}; k = {k1, k0}; flagged = triangles left to the
 * reference's edge functions alone.  For tests: it replaces no reference interface. */
int rts_tri_filter(const float* tri, int n_triangles, float* out, double* k, int32_t* flagged);

/* 8-bit RGB PNG (stbi_write_png in SaveFrame, src/core/Utility.h:19-30): width*height*3 bytes,
 * row 0 = top (rt_tonemap's output order).  Stored (uncompressed) deflate, no zlib needed. */
int rts_write_png(const char* path, int width, int height, const uint8_t* rgb);

#ifdef __cplusplus
}
#endif
#endif
