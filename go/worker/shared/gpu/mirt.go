// Package gpu is the cgo binding of libmirt (include/mirt.h) for the reference's Go
// workers: it replaces the per-pixel tracer.Trace loop of worker/distributed/main.go:67-89
// (and of worker/sequential/main.go:21-28) with one mirt_trace_tile call per work order.
//
// Uncompiled here: this image has no Go toolchain (go/README.md).  worker_c/mirt_worker.c
// runs the same call sequence in C against the built library, and tests/test_c_worker.py
// checks its frames bit for bit.
package gpu

// Where libmirt lives is the builder's environment, not this file's (INTEGRATION.md §cgo):
//
//	MIRT=/path/to/this/repo
//	CGO_CFLAGS="-I$MIRT/include" \
//	CGO_LDFLAGS="-L$MIRT/distributed_raytracer_amd -Wl,-rpath,$MIRT/distributed_raytracer_amd" \
//	go build ./worker/gpu

/*
#cgo LDFLAGS: -lmirt
#include <stdlib.h>
#include "mirt.h"
*/
import "C"

import (
	"context"
	"fmt"
	"math"
	"strings"
	"unsafe"

	"github.com/mwindels/distributed-raytracer/shared/state"
)

// Worker holds one libmirt context (one GPU), or one box (several GPUs behind one worker,
// mirt_box_*), and the meshes uploaded to it.
type Worker struct {
	ctx    *C.mirt_ctx
	box    *C.mirt_box
	meshes map[string]C.uint32_t // model path -> GPU mesh id
}

// Error is a failed libmirt call: the entry, its MIRT_E_* code and mirt_last_error().
type Error struct {
	Call string
	Code int
	Msg  string
}

func (e *Error) Error() string { return fmt.Sprintf("%s: %s (code %d)", e.Call, e.Msg, e.Code) }

// Transient reports whether retrying the call may succeed: the device or memory was
// unavailable.  A bad argument (a GPU index that does not exist), a library built for another
// GPU or a limit is permanent.
func (e *Error) Transient() bool {
	if e.Code == int(C.MIRT_E_NOMEM) {
		return true
	}
	return e.Code == int(C.MIRT_E_DEVICE) && !strings.Contains(e.Msg, "built for gfx950 only")
}

func lastError(call string, rc C.int) error {
	return &Error{Call: call, Code: int(rc), Msg: C.GoString(C.mirt_last_error())}
}

// DeviceCount is the number of HIP devices the process sees.
func DeviceCount() int { return int(C.mirt_device_count()) }

// New opens the GPU `device` (one worker process per GPU).
func New(device int) (*Worker, error) {
	w := &Worker{meshes: map[string]C.uint32_t{}}
	if rc := C.mirt_create(C.int(device), &w.ctx); rc != C.MIRT_OK {
		return nil, lastError("mirt_create", rc)
	}
	return w, nil
}

// NewBox opens one worker over several GPUs (mirt_box_create): every work order is cut into
// 8-pixel column strips dealt over the devices and assembled on the first (RCCL over xGMI),
// so a master sees ONE drop-in worker for the whole box.
func NewBox(devices []int) (*Worker, error) {
	if len(devices) == 0 {
		return nil, &Error{Call: "mirt_box_create", Code: int(C.MIRT_E_INVALID), Msg: "no devices"}
	}
	devs := (*C.int)(C.calloc(C.size_t(len(devices)), C.size_t(unsafe.Sizeof(C.int(0)))))
	defer C.free(unsafe.Pointer(devs))
	arr := unsafe.Slice(devs, len(devices))
	for i, d := range devices {
		arr[i] = C.int(d)
	}
	w := &Worker{meshes: map[string]C.uint32_t{}}
	if rc := C.mirt_box_create(devs, C.uint32_t(len(devices)), &w.box); rc != C.MIRT_OK {
		return nil, lastError("mirt_box_create", rc)
	}
	return w, nil
}

// Close releases the context (or box) and every mesh on it.
func (w *Worker) Close() {
	if w.ctx != nil {
		C.mirt_destroy(w.ctx)
		w.ctx = nil
	}
	if w.box != nil {
		C.mirt_box_destroy(w.box)
		w.box = nil
	}
}

// ReleaseMeshes frees every uploaded mesh: a worker that registers again may receive another
// scene.  The context (device workspaces, streams) stays open for the process's life.
func (w *Worker) ReleaseMeshes() {
	for path, id := range w.meshes {
		if w.box != nil {
			C.mirt_box_mesh_release(w.box, id)
		} else {
			C.mirt_mesh_release(w.ctx, id)
		}
		delete(w.meshes, path)
	}
}

// UploadScene uploads every mesh of the scene the master sent at registration
// (worker/distributed/main.go:115-126; shared/state/mesh.go:100-106).  Meshes are
// immutable for the worker's life: frames only carry EnvMutables diffs.
func (w *Worker) UploadScene(scene state.Environment) error {
	for path, m := range scene.MirtMeshes() {
		if err := w.uploadMesh(path, m); err != nil {
			return err
		}
	}
	return nil
}

func (w *Worker) uploadMesh(path string, m *state.Mesh) error {
	f := m.Flatten()
	if len(f.FMat) == 0 || len(f.V) == 0 {
		return fmt.Errorf("mesh %q has no faces", path)
	}
	// plain numeric arrays cross the boundary (no Go pointers inside): cgo-safe
	mats := make([]C.mirt_material, len(f.Mats))
	for i, mt := range f.Mats {
		ka, kd, ks := mt.Ka.Floats(), mt.Kd.Floats(), mt.Ks.Floats()
		for k := 0; k < 3; k++ {
			mats[i].ka[k], mats[i].kd[k], mats[i].ks[k] = C.double(ka[k]), C.double(kd[k]), C.double(ks[k])
		}
		mats[i].ns = C.double(mt.Ns)
	}
	var vn *C.double
	var fn *C.uint32_t
	if len(f.VN) > 0 {
		vn, fn = (*C.double)(unsafe.Pointer(&f.VN[0])), (*C.uint32_t)(unsafe.Pointer(&f.FN[0]))
	}
	var matp *C.mirt_material
	if len(mats) > 0 {
		matp = &mats[0]
	}
	var id C.uint32_t
	var rc C.int
	if w.box != nil {
		rc = C.mirt_box_mesh_upload(w.box, (*C.double)(unsafe.Pointer(&f.V[0])), C.uint32_t(len(f.V)/3), vn,
			C.uint32_t(len(f.VN)/3), (*C.uint32_t)(unsafe.Pointer(&f.FV[0])), fn,
			(*C.uint32_t)(unsafe.Pointer(&f.FMat[0])), C.uint32_t(len(f.FMat)), matp, C.uint32_t(len(mats)), &id)
	} else {
		rc = C.mirt_mesh_upload(w.ctx, (*C.double)(unsafe.Pointer(&f.V[0])), C.uint32_t(len(f.V)/3), vn,
			C.uint32_t(len(f.VN)/3), (*C.uint32_t)(unsafe.Pointer(&f.FV[0])), fn,
			(*C.uint32_t)(unsafe.Pointer(&f.FMat[0])), C.uint32_t(len(f.FMat)), matp, C.uint32_t(len(mats)), &id)
	}
	if rc != C.MIRT_OK {
		return lastError("mirt_mesh_upload", rc)
	}
	w.meshes[path] = id
	return nil
}

// frame builds a mirt_frame in C memory (it points at the object and light arrays, so it
// cannot live in Go memory under the cgo pointer rules); free releases it.
func (w *Worker) frame(scene state.Environment, env *state.EnvMutables) (fr *C.mirt_frame, free func(), err error) {
	objs := env.MirtObjects(scene)
	if len(objs) > C.MIRT_MAX_OBJECTS || len(env.Lights) > C.MIRT_MAX_LIGHTS {
		return nil, nil, fmt.Errorf("%d objects / %d lights: the GPU frame holds at most %d / %d",
			len(objs), len(env.Lights), C.MIRT_MAX_OBJECTS, C.MIRT_MAX_LIGHTS)
	}
	fr = (*C.mirt_frame)(C.calloc(1, C.size_t(unsafe.Sizeof(C.mirt_frame{}))))
	var cobj *C.mirt_object
	var clights *C.mirt_light
	if len(objs) > 0 {
		cobj = (*C.mirt_object)(C.calloc(C.size_t(len(objs)), C.size_t(unsafe.Sizeof(C.mirt_object{}))))
		arr := unsafe.Slice(cobj, len(objs))
		for i, o := range objs {
			id, ok := w.meshes[o.Path]
			if !ok {
				C.free(unsafe.Pointer(cobj))
				C.free(unsafe.Pointer(fr))
				return nil, nil, fmt.Errorf("object %d: mesh %q was not uploaded", i, o.Path)
			}
			arr[i].mesh_id = id
			arr[i].pos = [3]C.double{C.double(o.Pos.X), C.double(o.Pos.Y), C.double(o.Pos.Z)}
		}
		fr.objects, fr.n_objects = cobj, C.uint32_t(len(objs))
	}
	if len(env.Lights) > 0 {
		clights = (*C.mirt_light)(C.calloc(C.size_t(len(env.Lights)), C.size_t(unsafe.Sizeof(C.mirt_light{}))))
		arr := unsafe.Slice(clights, len(env.Lights))
		for i, l := range env.Lights {
			c := l.Col.Floats()
			arr[i].pos = [3]C.double{C.double(l.Pos.X), C.double(l.Pos.Y), C.double(l.Pos.Z)}
			arr[i].col = [3]C.double{C.double(c[0]), C.double(c[1]), C.double(c[2])}
		}
		fr.lights, fr.n_lights = clights, C.uint32_t(len(env.Lights))
	}
	// the camera exactly as tracer.go:15-22 uses it: Forward/Left/Up of state.NewCamera and
	// Go's own math.Tan(Fov/2) (tracer.go:17)
	cam := env.Cam
	f, l, u := cam.Forward(), cam.Left(), cam.Up()
	fr.camera.pos = [3]C.double{C.double(cam.Pos.X), C.double(cam.Pos.Y), C.double(cam.Pos.Z)}
	fr.camera.forward = [3]C.double{C.double(f.X), C.double(f.Y), C.double(f.Z)}
	fr.camera.left = [3]C.double{C.double(l.X), C.double(l.Y), C.double(l.Z)}
	fr.camera.up = [3]C.double{C.double(u.X), C.double(u.Y), C.double(u.Z)}
	fr.camera.fov = C.double(cam.Fov)
	fr.camera.proj_half_width = C.double(math.Tan(cam.Fov / 2.0))
	fr.max_bounces = 0 // the reference's Trace (reflections are a libmirt extension)
	free = func() {
		C.free(unsafe.Pointer(cobj))
		C.free(unsafe.Pointer(clights))
		C.free(unsafe.Pointer(fr))
	}
	return fr, free, nil
}

// BulkTrace traces the work-order rectangle (x, y, width, height) of a screenW x screenH
// screen: the loop of worker/distributed/main.go:67-89 in one call.  It returns
// width*height*3 bytes, pixel (i, j) at 3*(i*height + j): the results[i*height + j]
// layout and uint8(255*c) truncation of main.go:79-86 (misses are black).  A cancelled
// ctx makes the call return MIRT_E_CANCELLED between kernel launches, as main.go:73
// checks ctx.Err() per pixel.
func (w *Worker) BulkTrace(ctx context.Context, scene state.Environment, env *state.EnvMutables, x, y, width, height,
	screenW, screenH int) ([]uint8, error) {
	fr, free, err := w.frame(scene, env)
	if err != nil {
		return nil, err
	}
	defer free()
	n := width * height
	if n == 0 {
		return nil, nil
	}
	rgb8 := (*C.uint8_t)(C.malloc(C.size_t(3 * n)))
	defer C.free(unsafe.Pointer(rgb8))
	cc := (*C.int)(C.calloc(1, C.size_t(unsafe.Sizeof(C.int(0)))))
	defer C.free(unsafe.Pointer(cc))
	done := make(chan struct{})
	defer close(done)
	go func() { // the cancel flag lives in C memory (cgo: C never holds Go pointers)
		select {
		case <-ctx.Done():
			*(*C.int)(unsafe.Pointer(cc)) = 1
		case <-done:
		}
	}()
	out := C.mirt_outputs{rgb8: rgb8}
	var rc C.int
	if w.box != nil { // the order over every GPU of the box
		rc = C.mirt_box_trace_tile(w.box, fr, C.uint32_t(x), C.uint32_t(y), C.uint32_t(width), C.uint32_t(height),
			C.uint32_t(screenW), C.uint32_t(screenH), &out, cc, nil)
	} else {
		rc = C.mirt_trace_tile(w.ctx, fr, C.uint32_t(x), C.uint32_t(y), C.uint32_t(width), C.uint32_t(height),
			C.uint32_t(screenW), C.uint32_t(screenH), &out, cc, nil)
	}
	if rc != C.MIRT_OK {
		return nil, lastError("mirt_trace_tile", rc)
	}
	return C.GoBytes(unsafe.Pointer(rgb8), C.int(3*n)), nil
}
