// gob.cpp — Go encoding/gob stream decoder for the reference's wire state (gob.hpp).
//
// Wire format (the encoding/gob package documentation, Go standard library):
//   stream   = message*;  message = uint(length) payload
//   payload  = int(-id) wireType            a type definition
//            | int(id) value                a value (non-struct values: uint(0) first)
//   uint     = one byte < 128, or byte(-n) then n big-endian bytes
//   int      = uint u: u >> 1, complemented when u & 1
//   float    = uint of the byte-reversed IEEE-754 bits
//   string, []byte = uint(len) bytes;   bool = uint 0/1
//   struct   = (uint(field delta) field)* uint(0); fields with zero values are omitted
//   slice, array = uint(count) elem*;   map = uint(count) (key elem)*
//   interface = uint(len) name; then int(id) uint(len) value of the concrete type
//   GobEncoder / BinaryMarshaler types = uint(len) bytes (their own format)
// Predefined type ids: bool 1, int 2, uint 3, float 4, []byte 5, string 6, complex 7,
// interface 8, wireType 16, arrayType 17, CommonType 18, sliceType 19, structType 20,
// fieldType 21, []fieldType 22, mapType 23; user types from 65.
#include "gob.hpp"

#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <map>
#include <memory>

namespace mirt {
namespace gob {
namespace {

struct Bad {
    std::string msg;
};
[[noreturn]] void bad(const std::string& m) { throw Bad{m}; }

enum : int64_t {
    tBool = 1, tInt = 2, tUint = 3, tFloat = 4, tBytes = 5, tString = 6, tComplex = 7, tInterface = 8,
};
constexpr int kMaxDepth = 64;

struct WireType {
    enum Kind { Array, Slice, Struct, Map, External } kind = Struct;
    std::string name;
    int64_t elem = 0, key = 0, len = 0;
    std::vector<std::pair<std::string, int64_t>> fields;  // Struct
};

struct Value {
    enum Kind { None, Bool, Int, Uint, Float, Bytes, Complex, List, Map, Struct, Iface, External } kind = None;
    uint64_t u = 0;
    int64_t i = 0;
    double f = 0, f2 = 0;
    std::string bytes;          // Bytes (strings too), External payload, Iface: concrete type name
    std::vector<Value> items;   // List; Map: key, elem alternating; Struct: per field; Iface: the value
    const WireType* type = nullptr;  // Struct

    // field of a struct by name (gob matches fields by name); nullptr when absent (zero)
    const Value* field(const char* name) const {
        if (kind != Struct || !type) return nullptr;
        for (size_t k = 0; k < type->fields.size() && k < items.size(); ++k)
            if (type->fields[k].first == name) return items[k].kind == None ? nullptr : &items[k];
        return nullptr;
    }
};

// A cursor over one message (or any byte range).
struct Reader {
    const uint8_t* p;
    const uint8_t* e;
    bool done() const { return p == e; }
    uint8_t byte() {
        if (p >= e) bad("truncated gob data");
        return *p++;
    }
    uint64_t u() {
        const uint8_t b = byte();
        if (b < 0x80) return b;
        const int n = 256 - b;  // byte(-n)
        if (n > 8) bad("gob uint longer than 8 bytes");
        uint64_t x = 0;
        for (int k = 0; k < n; ++k) x = (x << 8) | byte();
        return x;
    }
    int64_t i() {
        const uint64_t x = u();
        return (x & 1) ? ~(int64_t)(x >> 1) : (int64_t)(x >> 1);
    }
    double f() {
        uint64_t x = u(), r = 0;
        for (int k = 0; k < 8; ++k) {  // byte-reversed IEEE-754 bits
            r = (r << 8) | (x & 0xff);
            x >>= 8;
        }
        double d;
        memcpy(&d, &r, 8);
        return d;
    }
    size_t count() {  // a length or element count: bounded by the bytes left
        const uint64_t n = u();
        if (n > (uint64_t)(e - p)) bad("gob count exceeds the data left");
        return (size_t)n;
    }
    std::string str() {
        const size_t n = count();
        std::string s((const char*)p, n);
        p += n;
        return s;
    }
    Reader sub(size_t n) {
        if (n > (size_t)(e - p)) bad("truncated gob data");
        Reader r{p, p + n};
        p += n;
        return r;
    }
};

// Walk one encoded struct: on_field(field number, reader) per transmitted field.
template <typename F>
void walk_struct(Reader& m, F on_field) {
    int64_t fn = -1;
    for (;;) {
        const uint64_t d = m.u();
        if (d == 0) return;
        if (d > 1024) bad("gob field delta out of range");
        fn += (int64_t)d;
        on_field(fn);
    }
}

struct Stream {
    Reader r;
    std::map<int64_t, std::unique_ptr<WireType>> types;
    int depth = 0;

    explicit Stream(const uint8_t* data, size_t n) : r{data, data + n} {}

    // a negative type id introduces a definition; INT64_MIN has no positive counterpart
    static int64_t defined_id(int64_t id) {
        if (id == INT64_MIN) bad("gob type id out of range");
        return -id;
    }

    // --- type definitions: a wireType value (encoding/gob type.go wireType and its parts)
    void common(Reader& m, WireType& t) {  // CommonType{Name string; Id int}
        walk_struct(m, [&](int64_t f) {
            if (f == 0) t.name = m.str();
            else if (f == 1) (void)m.i();
            else bad("bad CommonType field");
        });
    }
    WireType wire_type(Reader& m) {
        WireType t;
        bool seen = false;
        walk_struct(m, [&](int64_t f) {
            if (seen) bad("wireType with two kinds");
            seen = true;
            switch (f) {
                case 0:  // ArrayT *arrayType{CommonType; Elem typeId; Len int}
                    t.kind = WireType::Array;
                    walk_struct(m, [&](int64_t g) {
                        if (g == 0) common(m, t);
                        else if (g == 1) t.elem = m.i();
                        else if (g == 2) t.len = m.i();
                        else bad("bad arrayType field");
                    });
                    break;
                case 1:  // SliceT *sliceType{CommonType; Elem typeId}
                    t.kind = WireType::Slice;
                    walk_struct(m, [&](int64_t g) {
                        if (g == 0) common(m, t);
                        else if (g == 1) t.elem = m.i();
                        else bad("bad sliceType field");
                    });
                    break;
                case 2:  // StructT *structType{CommonType; Field []*fieldType{Name string; Id typeId}}
                    t.kind = WireType::Struct;
                    walk_struct(m, [&](int64_t g) {
                        if (g == 0) {
                            common(m, t);
                        } else if (g == 1) {
                            const size_t n = m.count();
                            for (size_t k = 0; k < n; ++k) {
                                std::pair<std::string, int64_t> fd;
                                walk_struct(m, [&](int64_t h) {
                                    if (h == 0) fd.first = m.str();
                                    else if (h == 1) fd.second = m.i();
                                    else bad("bad fieldType field");
                                });
                                t.fields.push_back(fd);
                            }
                        } else {
                            bad("bad structType field");
                        }
                    });
                    break;
                case 3:  // MapT *mapType{CommonType; Key, Elem typeId}
                    t.kind = WireType::Map;
                    walk_struct(m, [&](int64_t g) {
                        if (g == 0) common(m, t);
                        else if (g == 1) t.key = m.i();
                        else if (g == 2) t.elem = m.i();
                        else bad("bad mapType field");
                    });
                    break;
                case 4: case 5: case 6:  // GobEncoderT / BinaryMarshalerT / TextMarshalerT
                    t.kind = WireType::External;
                    walk_struct(m, [&](int64_t g) {
                        if (g == 0) common(m, t);
                        else bad("bad gobEncoderType field");
                    });
                    break;
                default:
                    bad("unknown wireType kind");
            }
        });
        if (!seen) bad("empty wireType");
        return t;
    }
    void define(Reader& m, int64_t id) {
        if (id < 65) bad("gob type definition for a predefined id");
        if (types.count(id)) bad("gob type redefined");
        types[id].reset(new WireType(wire_type(m)));
    }
    const WireType& type(int64_t id) {
        auto it = types.find(id);
        if (it == types.end()) bad("gob value of an undefined type id " + std::to_string(id));
        return *it->second;
    }

    // --- values
    Value value(Reader& m, int64_t id) {
        if (++depth > kMaxDepth) bad("gob value nested too deeply");
        Value v;
        switch (id) {
            case tBool: v.kind = Value::Bool; v.u = m.u(); break;
            case tInt: v.kind = Value::Int; v.i = m.i(); break;
            case tUint: v.kind = Value::Uint; v.u = m.u(); break;
            case tFloat: v.kind = Value::Float; v.f = m.f(); break;
            case tBytes: case tString: v.kind = Value::Bytes; v.bytes = m.str(); break;
            case tComplex: v.kind = Value::Complex; v.f = m.f(); v.f2 = m.f(); break;
            case tInterface: v = iface(m); break;
            default: {
                const WireType& t = type(id);
                switch (t.kind) {
                    case WireType::Array:
                    case WireType::Slice: {
                        const size_t n = m.count();
                        if (t.kind == WireType::Array && (int64_t)n != t.len) bad("gob array length mismatch");
                        v.kind = Value::List;
                        v.items.reserve(n);
                        for (size_t k = 0; k < n; ++k) v.items.push_back(value(m, t.elem));
                        break;
                    }
                    case WireType::Map: {
                        const size_t n = m.count();
                        v.kind = Value::Map;
                        for (size_t k = 0; k < n; ++k) {
                            v.items.push_back(value(m, t.key));
                            v.items.push_back(value(m, t.elem));
                        }
                        break;
                    }
                    case WireType::Struct: v = structure(m, t); break;
                    case WireType::External: v.kind = Value::External; v.bytes = m.str(); break;
                }
            }
        }
        --depth;
        return v;
    }
    Value structure(Reader& m, const WireType& t) {
        Value v;
        v.kind = Value::Struct;
        v.type = &t;
        v.items.resize(t.fields.size());
        walk_struct(m, [&](int64_t f) {
            if (f >= (int64_t)t.fields.size()) bad("gob struct field out of range");
            v.items[f] = value(m, t.fields[f].second);
        });
        return v;
    }
    // A value of a type id as the top of a message or of an interface: structs as
    // themselves, anything else as a singleton (field delta 0 first).
    Value top(Reader& m, int64_t id) {
        if (id >= 65 && type(id).kind == WireType::Struct) return structure(m, type(id));
        if (m.u() != 0) bad("gob singleton with a non-zero field delta");
        return value(m, id);
    }
    Value iface(Reader& m) {
        Value v;
        v.kind = Value::Iface;
        v.bytes = m.str();       // the concrete type's registered name; empty: nil interface
        if (v.bytes.empty()) return v;
        int64_t id = m.i();
        while (id < 0) {  // a type definition inside the value (encoding/gob decodeTypeSequence)
            define(m, defined_id(id));
            if (!m.done()) (void)m.u();
            id = m.i();
        }
        Reader body = m.sub(m.count());
        v.items.push_back(top(body, id));
        if (!body.done()) bad("extra data in a gob interface value");
        return v;
    }

    // The next top-level value of the stream (type definitions before it are absorbed).
    Value next() {
        for (;;) {
            if (r.done()) bad("gob stream ended before the expected value");
            Reader m = r.sub(r.count());
            const int64_t id = m.i();
            if (id < 0) {
                define(m, defined_id(id));
                if (!m.done()) bad("extra data after a gob type definition");
                continue;
            }
            Value v = top(m, id);
            if (!m.done()) bad("extra data in a gob message");
            return v;
        }
    }
};

// ------------------------------------------------------------------ the reference's shapes
const Value& want(const Value& v, Value::Kind k, const char* what) {
    if (v.kind != k) bad(std::string("unexpected gob value for ") + what);
    return v;
}
double fnum(const Value* v) {  // absent (zero) or float
    if (!v) return 0.0;
    if (v->kind != Value::Float) bad("expected a float64");
    return v->f;
}
uint64_t unum(const Value& v, const char* what) {
    if (v.kind != Value::Uint) bad(std::string("expected a uint for ") + what);
    return v.u;
}
void vector3(const Value* v, double out[3]) {  // geom.Vector{X, Y, Z float64} (vector.go:7-11)
    if (!v) {
        out[0] = out[1] = out[2] = 0.0;
        return;
    }
    want(*v, Value::Struct, "geom.Vector");
    out[0] = fnum(v->field("X"));
    out[1] = fnum(v->field("Y"));
    out[2] = fnum(v->field("Z"));
}
// colour.RGB: three uint8 values (colour.go:63-83); NewRGB(u8) = u8 / 255 (colour.go:28-30).
// An absent (zero) RGB field decodes as {0, 0, 0}.
void rgb(const Value* v, double out[3]) {
    if (!v) {
        out[0] = out[1] = out[2] = 0.0;
        return;
    }
    const std::string& p = want(*v, Value::External, "colour.RGB").bytes;
    Stream s((const uint8_t*)p.data(), p.size());
    for (int k = 0; k < 3; ++k) {
        const uint64_t c = unum(s.next(), "a colour channel");
        if (c > 255) bad("colour channel above 255");
        out[k] = (double)c / 255.0;
    }
}
std::string payload(const Value& v, const char* what) { return want(v, Value::External, what).bytes; }
// The concrete value inside an interface element of a []rtreego.Spatial.
const Value& spatial(const Value& v, const char* what) {
    want(v, Value::Iface, what);
    if (v.items.empty()) bad(std::string("nil ") + what);
    return v.items[0];
}

Mesh mesh(const std::string& p) {  // Mesh.UnmarshalBinary (mesh.go:238-272)
    Stream s((const uint8_t*)p.data(), p.size());
    Mesh m;
    const Value verts = s.next(), norms = s.next(), faces = s.next(), mats = s.next();
    for (const Value& x : want(verts, Value::List, "Mesh.vertices").items) {
        double a[3];
        vector3(&x, a);
        m.v.insert(m.v.end(), a, a + 3);
    }
    for (const Value& x : want(norms, Value::List, "Mesh.vertexNormals").items) {
        double a[3];
        vector3(&x, a);
        m.vn.insert(m.vn.end(), a, a + 3);
    }
    for (const Value& x : want(faces, Value::List, "Mesh faces").items) {
        const std::string fp = payload(spatial(x, "face"), "face");  // face.UnmarshalBinary (mesh.go:73-91)
        Stream fs((const uint8_t*)fp.data(), fp.size());
        const Value vi = fs.next(), ni = fs.next(), mi = fs.next();
        for (const Value* a : {&vi, &ni}) {
            if (want(*a, Value::List, "face indices").items.size() != 3) bad("face index array is not [3]uint");
            for (const Value& k : a->items) (a == &vi ? m.fv : m.fn).push_back(unum(k, "a face index"));
        }
        m.fmat.push_back(unum(mi, "a face material"));
    }
    for (const Value& x : want(mats, Value::List, "Mesh.materials").items) {
        want(x, Value::Struct, "Material");
        mirt_material mm;
        rgb(x.field("Ka"), mm.ka);
        rgb(x.field("Kd"), mm.kd);
        rgb(x.field("Ks"), mm.ks);
        mm.ns = fnum(x.field("Ns"));
        m.mats.push_back(mm);
    }
    const uint64_t nv = m.v.size() / 3, nn = m.vn.size() / 3, nm = m.mats.size();
    for (size_t k = 0; k < m.fmat.size(); ++k) {
        for (int c = 0; c < 3; ++c) {
            if (m.fv[3 * k + c] >= nv) bad("face vertex index out of range");
            if (nn && m.fn[3 * k + c] >= nn) bad("face normal index out of range");
        }
        if (m.fmat[k] >= nm) bad("face material index out of range");
    }
    return m;
}

// Diagnostic JSON rendering of a decoded value (floats keep a '.', so -0 stays a float;
// NaN / Infinity as the common JSON extension).
void jfloat(double f, std::string& o) {
    if (f != f) {
        o += "NaN";
        return;
    }
    if (f == __builtin_inf() || f == -__builtin_inf()) {
        o += f > 0 ? "Infinity" : "-Infinity";
        return;
    }
    char buf[40];
    snprintf(buf, sizeof buf, "%.17g", f);
    o += buf;
    if (!strpbrk(buf, ".e")) o += ".0";
}
void json(const Value& v, std::string& o) {
    char buf[64];
    switch (v.kind) {
        case Value::None: o += "null"; break;
        case Value::Bool: o += v.u ? "true" : "false"; break;
        case Value::Int: o += std::to_string(v.i); break;
        case Value::Uint: o += std::to_string(v.u); break;
        case Value::Float: jfloat(v.f, o); break;
        case Value::Complex:
            o += '[';
            jfloat(v.f, o);
            o += ", ";
            jfloat(v.f2, o);
            o += ']';
            break;
        case Value::Bytes:
            o += '"';
            for (unsigned char c : v.bytes) {
                if (c == '"' || c == '\\') {
                    o += '\\';
                    o += (char)c;
                } else if (c < 0x20 || c >= 0x7f) {
                    snprintf(buf, sizeof buf, "\\u%04x", c);
                    o += buf;
                } else {
                    o += (char)c;
                }
            }
            o += '"';
            break;
        case Value::External:
            o += "{\"$ext\": \"";
            for (unsigned char c : v.bytes) {
                snprintf(buf, sizeof buf, "%02x", c);
                o += buf;
            }
            o += "\"}";
            break;
        case Value::Iface: {
            if (v.items.empty()) {
                o += "null";
                break;
            }
            Value name;
            name.kind = Value::Bytes;
            name.bytes = v.bytes;
            o += "{\"$type\": ";
            json(name, o);
            o += ", \"$value\": ";
            json(v.items[0], o);
            o += "}";
            break;
        }
        case Value::List:
        case Value::Map:
            o += '[';
            for (size_t k = 0; k < v.items.size(); k += (v.kind == Value::Map ? 2 : 1)) {
                if (k) o += ", ";
                if (v.kind == Value::Map) {
                    o += '[';
                    json(v.items[k], o);
                    o += ", ";
                    json(v.items[k + 1], o);
                    o += ']';
                } else {
                    json(v.items[k], o);
                }
            }
            o += ']';
            break;
        case Value::Struct: {
            o += '{';
            bool first = true;
            for (size_t k = 0; k < v.items.size(); ++k) {
                if (v.items[k].kind == Value::None) continue;
                Value name;
                name.kind = Value::Bytes;
                name.bytes = v.type->fields[k].first;
                if (!first) o += ", ";
                first = false;
                json(name, o);
                o += ": ";
                json(v.items[k], o);
            }
            o += '}';
            break;
        }
    }
}

}  // namespace

bool to_json(const uint8_t* data, size_t n, std::string& out, std::string& err) {
    try {
        Stream s(data, n);
        out = "[";
        bool first = true;
        while (!s.r.done()) {
            if (!first) out += ", ";
            first = false;
            json(s.next(), out);
        }
        out += "]";
        return true;
    } catch (const Bad& b) {
        err = "gob: " + b.msg;
        return false;
    } catch (const std::exception& e) {
        err = std::string("gob: ") + e.what();
        return false;
    }
}

bool decode_environment(const uint8_t* data, size_t n, Immutables& out, std::string& err) {
    try {
        out = Immutables();
        Stream s0(data, n);  // gob(state.Environment) -> Environment.MarshalBinary bytes
        const std::string env = payload(s0.next(), "state.Environment");
        Stream s1((const uint8_t*)env.data(), env.size());  // gob(envImmutables)
        const std::string imm = payload(s1.next(), "envImmutables");
        Stream s2((const uint8_t*)imm.data(), imm.size());  // envImmutables.MarshalBinary
        const Value meshes = s2.next(), paths = s2.next();
        const auto& mi = want(meshes, Value::Map, "envImmutables.meshes").items;
        for (size_t k = 0; k + 1 < mi.size(); k += 2)
            out.meshes.emplace_back(want(mi[k], Value::Bytes, "a model path").bytes,
                                    mesh(payload(mi[k + 1], "state.Mesh")));
        const auto& pi = want(paths, Value::Map, "envImmutables.paths").items;
        for (size_t k = 0; k + 1 < pi.size(); k += 2)
            out.paths.emplace_back(unum(pi[k], "an object id"), want(pi[k + 1], Value::Bytes, "a model path").bytes);
        return true;
    } catch (const Bad& b) {
        err = "gob Environment: " + b.msg;
        return false;
    } catch (const std::exception& e) {
        err = std::string("gob Environment: ") + e.what();
        return false;
    }
}

bool decode_mutables(const uint8_t* data, size_t n, Mutables& out, std::string& err) {
    try {
        out = Mutables();
        Stream s0(data, n);  // gob(state.EnvMutables) -> EnvMutables.MarshalBinary bytes
        const std::string mut = payload(s0.next(), "state.EnvMutables");
        Stream s((const uint8_t*)mut.data(), mut.size());  // EnvMutables.UnmarshalBinary (environment.go:120-146)
        const Value objs = s.next(), lights = s.next(), cam = s.next();
        for (const Value& x : want(objs, Value::List, "EnvMutables objects").items) {
            const std::string op = payload(spatial(x, "Object"), "Object");  // Object.UnmarshalBinary (object.go:129-148)
            Stream os((const uint8_t*)op.data(), op.size());
            const Value pos = os.next(), id = os.next();
            Object ob;
            vector3(&pos, ob.pos);
            ob.id = unum(id, "Object.id");
            out.objects.push_back(ob);
        }
        for (const Value& x : want(lights, Value::List, "EnvMutables.Lights").items) {
            want(x, Value::Struct, "Light");
            mirt_light lt;
            vector3(x.field("Pos"), lt.pos);
            rgb(x.field("Col"), lt.col);
            out.lights.push_back(lt);
        }
        const std::string cp = payload(cam, "Camera");  // Camera.UnmarshalBinary (camera.go:177-203)
        Stream cs((const uint8_t*)cp.data(), cp.size());
        const Value pos = cs.next(), fwd = cs.next(), fov = cs.next();
        vector3(&pos, out.cam_pos);
        vector3(&fwd, out.cam_forward);
        out.fov = want(fov, Value::Float, "Camera fov").f;
        return true;
    } catch (const Bad& b) {
        err = "gob EnvMutables: " + b.msg;
        return false;
    } catch (const std::exception& e) {
        err = std::string("gob EnvMutables: ") + e.what();
        return false;
    }
}

}  // namespace gob
}  // namespace mirt
