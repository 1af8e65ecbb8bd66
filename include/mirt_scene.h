/*
 * mirt_scene.h — C++ host-side restatement of the reference's scene loader, exported
 * as plain C from libmirt.so.  Replaces, for a non-Go caller (C++ harness, Python):
 *   shared/state/environment.go:162-234  EnvironmentFromFile
 *   shared/state/mesh.go:109-213         MeshFromFile (gwob OBJ/MTL semantics assumed:
 *                                        float32 coordinates, fan triangulation)
 *   shared/state/camera.go:35-44         NewCamera
 * A Go worker keeps its own loader (north star) and passes the arrays to
 * mirt_mesh_upload directly; see INTEGRATION.md.
 */
#ifndef MIRT_SCENE_H
#define MIRT_SCENE_H

#include "mirt.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mirt_scene mirt_scene;

/* One loaded mesh, arrays owned by the scene (valid until mirt_scene_free). */
typedef struct {
    const double *vertices;  uint32_t n_vertices;
    const double *normals;   uint32_t n_normals;
    const uint32_t *face_v;  const uint32_t *face_n;  const uint32_t *face_mat;
    uint32_t n_faces;
    const mirt_material *materials; uint32_t n_materials;
} mirt_mesh_view;

int mirt_scene_load(const char *path, mirt_scene **out);
void mirt_scene_free(mirt_scene *s);
/* detail of the last mirt_scene_load failure on this thread */
const char *mirt_scene_last_error(void);
uint32_t mirt_scene_mesh_count(const mirt_scene *s);
int mirt_scene_mesh(const mirt_scene *s, uint32_t i, mirt_mesh_view *out);
uint32_t mirt_scene_object_count(const mirt_scene *s);
/* object i: mesh index into the scene's meshes, and position */
int mirt_scene_object(const mirt_scene *s, uint32_t i, mirt_object *out);
uint32_t mirt_scene_light_count(const mirt_scene *s);
int mirt_scene_light(const mirt_scene *s, uint32_t i, mirt_light *out);
/* camera from the JSON via NewCamera + Go math.Tan */
int mirt_scene_camera(const mirt_scene *s, mirt_camera *out);

#ifdef __cplusplus
}
#endif
#endif /* MIRT_SCENE_H */
