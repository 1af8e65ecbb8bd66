// export_mirt.go — accessors the GPU worker needs from package state (new file in the
// reference's shared/state; nothing else in the package changes).  Uncompiled here: this
// image has no Go toolchain (see go/README.md).
package state

import (
	"github.com/mwindels/distributed-raytracer/shared/geom"
	"github.com/mwindels/rtreego"
)

// MirtMesh is a mesh flattened for libmirt's mirt_mesh_upload (include/mirt.h): xyz per
// vertex and vertex normal, and per face its three vertex indices, three vertex-normal
// indices and material index (shared/state/mesh.go:21-27, 100-106).
type MirtMesh struct {
	V, VN        []float64
	FV, FN, FMat []uint32
	Mats         []Material
}

// Flatten lists the faces in the order Object.Intersection visits them
// (shared/state/object.go:76: the R-tree's SearchCondition order); the GPU breaks exact
// distance ties by this order.
func (m *Mesh) Flatten() MirtMesh {
	var out MirtMesh
	for _, p := range m.vertices {
		out.V = append(out.V, p.X, p.Y, p.Z)
	}
	for _, n := range m.vertexNormals {
		out.VN = append(out.VN, n.X, n.Y, n.Z)
	}
	for _, s := range m.faces.SearchCondition(func(*rtreego.Rect) bool { return true }) {
		f := s.(face)
		out.FV = append(out.FV, uint32(f.verts[0]), uint32(f.verts[1]), uint32(f.verts[2]))
		out.FN = append(out.FN, uint32(f.vertNorms[0]), uint32(f.vertNorms[1]), uint32(f.vertNorms[2]))
		out.FMat = append(out.FMat, uint32(f.mat))
	}
	out.Mats = m.materials
	return out
}

// MirtMeshes maps each model path of the environment to its mesh (environment.go:24-27).
func (e Environment) MirtMeshes() map[string]*Mesh {
	return e.immutable.meshes
}

// MirtObject is one object of a frame: its mesh's path and its position.
type MirtObject struct {
	Path string
	Pos  geom.Vector
}

// MirtObjects lists the frame's objects in the order tracer.trace visits them
// (worker/shared/tracer/tracer.go:32: the R-tree's SearchCondition order), resolving each
// object's mesh through the immutable part of e (environment.go:73-89 LinkTo).
func (em *EnvMutables) MirtObjects(e Environment) []MirtObject {
	var out []MirtObject
	for _, s := range em.Objs.SearchCondition(func(*rtreego.Rect) bool { return true }) {
		o := s.(*Object)
		out = append(out, MirtObject{Path: e.immutable.paths[o.id], Pos: o.Pos})
	}
	return out
}
