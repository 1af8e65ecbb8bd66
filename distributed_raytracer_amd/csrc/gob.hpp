// gob.hpp — decoder of the reference's network state (Go encoding/gob), host side.
//
// What the wire carries (reference paths):
//   MasterState.state (comms.proto:13-17), the Register reply
//     = gob(state.Environment)                      environment.go:236-249 (BinaryMarshaler)
//       -> gob(envImmutables)                       environment.go:30-45   (BinaryMarshaler)
//          -> map[string]*Mesh, map[uint]string     meshes by model path, object id -> path
//             Mesh -> []Vector, []Vector, []Spatial(face), []Material    mesh.go:215-236
//             face -> [3]uint, [3]uint, uint                             mesh.go:52-71
//             Material{Ka, Kd, Ks colour.RGB; Ns float64}                mesh.go:93-97
//             colour.RGB -> uint8, uint8, uint8 (uint8(255 c), truncated) colour.go:63-83
//   WorkOrder.diff (comms.proto:25-31), every BulkTrace
//     = gob(state.EnvMutables)                      environment.go:100-118 (BinaryMarshaler)
//       -> []Spatial(Object), []Light, Camera
//          Object -> Vector, uint (id)               object.go:112-127
//          Light{Pos Vector; Col colour.RGB}         light.go:10-13
//          Camera -> Vector pos, Vector forward, float64 fov   camera.go:156-174
// The decoder is generic over the gob stream (type definitions, structs matched by field
// name, zero fields omitted, interface values by registered name) and then reads these
// shapes; the receiving side's UnmarshalBinary rules are applied by the caller
// (scene.cpp): NewRGB(u8) = u8 / 255, NewCamera(pos, forward, fov), LinkTo by id.
#pragma once

#include <stdint.h>

#include <string>
#include <utility>
#include <vector>

#include "../../include/mirt.h"

namespace mirt {
namespace gob {

struct Mesh {
    std::vector<double> v, vn;  // vertices, vertex normals (already normalised by the sender)
    std::vector<uint64_t> fv, fn, fmat;  // per face: 3 vertex, 3 normal indices, material index
    std::vector<mirt_material> mats;     // colour channels as NewRGB(u8) = u8 / 255
};

struct Immutables {
    std::vector<std::pair<std::string, Mesh>> meshes;     // model path -> mesh (wire order)
    std::vector<std::pair<uint64_t, std::string>> paths;  // object id -> model path
};

struct Object {
    double pos[3];
    uint64_t id;
};

struct Mutables {
    std::vector<Object> objects;    // wire order (the sender's R-tree order)
    std::vector<mirt_light> lights;  // col = NewRGB(u8)
    double cam_pos[3], cam_forward[3], fov;
};

// Each returns false with a message in err on malformed or unexpected data.
bool decode_environment(const uint8_t* data, size_t n, Immutables& out, std::string& err);
bool decode_mutables(const uint8_t* data, size_t n, Mutables& out, std::string& err);
// Diagnostic: every top-level value of a gob stream as JSON (structs as objects of the
// fields transmitted, maps as [key, value] pairs, interfaces as {"$type", "$value"},
// GobEncoder / BinaryMarshaler payloads as {"$ext": hex}).
bool to_json(const uint8_t* data, size_t n, std::string& out, std::string& err);

}  // namespace gob
}  // namespace mirt
