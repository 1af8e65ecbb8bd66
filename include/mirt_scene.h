/*
 * mirt_scene.h — C++ host-side restatement of the reference's scene loader, exported
 * as plain C from libmirt.so.  Replaces, for a non-Go caller (C++ harness, Python):
 *   shared/state/environment.go:162-234  EnvironmentFromFile
 *   shared/state/mesh.go:109-213         MeshFromFile (gwob OBJ/MTL semantics assumed:
 *                                        float32 coordinates, fan triangulation)
 *   shared/state/camera.go:35-44         NewCamera
 * and the network state a worker receives (Go encoding/gob, decoded in csrc/gob.cpp):
 *   worker/distributed/main.go:118-126   Register: MasterState.state = gob(Environment)
 *                                        (environment.go:236-268, :30-62; mesh.go:215-272)
 *   worker/distributed/main.go:56-64     BulkTrace: WorkOrder.diff = gob(EnvMutables) and
 *                                        LinkTo (environment.go:73-146; object.go:112-148;
 *                                        camera.go:156-203; colour.go:63-107)
 * A Go worker keeps its own loader and gob (north star) and passes the arrays to
 * mirt_mesh_upload directly; see INTEGRATION.md.  A non-Go worker uses these.
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
/* camera from the JSON (or the gob diff) via NewCamera + Go math.Tan; MIRT_E_INVALID for a
 * scene that has none (mirt_scene_from_gob before linking) */
int mirt_scene_camera(const mirt_scene *s, mirt_camera *out);

/* mirt_object.mesh_id of an object whose id links to no mesh (LinkTo leaves its mesh nil,
 * environment.go:80-88; such an object is never hit, object.go:73-74: drop it from frames) */
#define MIRT_NO_MESH 0xffffffffu
/*
 * Register (worker/distributed/main.go:118-126): decode MasterState.state, the gob stream of
 * a state.Environment, into a scene holding the environment's meshes (in model-path order)
 * and its object id -> mesh links.  It has no objects, lights or camera.  MIRT_E_IO (detail
 * in mirt_scene_last_error) on malformed data or out-of-range face indices.
 */
int mirt_scene_from_gob(const uint8_t *state, size_t n, mirt_scene **out);
/*
 * BulkTrace (worker/distributed/main.go:56-64): decode WorkOrder.diff, the gob stream of a
 * state.EnvMutables, and link it to env (EnvMutables.LinkTo): a NEW scene that shares env's
 * meshes and holds the frame's objects (wire order; mesh_id = the linked mesh index or
 * MIRT_NO_MESH), lights (Col = NewRGB(u8)) and camera (NewCamera(pos, forward, fov), as
 * Camera.UnmarshalBinary rebuilds it; MIRT_E_CAMERA if that fails).  env is not modified,
 * so concurrent calls on one env are safe.  Free the result with mirt_scene_free.
 */
int mirt_scene_link_gob(const mirt_scene *env, const uint8_t *diff, size_t n, mirt_scene **out);
/* Diagnostic: the top-level values of any gob stream as a JSON array (structs: the fields
 * transmitted; maps: [key, value] pairs; interfaces: {"$type", "$value"}; GobEncoder /
 * BinaryMarshaler payloads: {"$ext": hex}).  *len = the JSON length; up to cap - 1 bytes
 * and a NUL are written to out (out may be NULL).  MIRT_E_IO on malformed data. */
int mirt_gob_json(const uint8_t *data, size_t n, char *out, size_t cap, size_t *len);

#ifdef __cplusplus
}
#endif
#endif /* MIRT_SCENE_H */
