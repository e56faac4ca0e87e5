// gltf.cpp -- stage 1 of the reference (src/stage1.zig): glTF 2.0 / GLB scene
// load into the flat triangle soup + material table the render seam takes.
//
//   loadGltfFile      stage1.zig:75-110   .gltf + external/data-URI buffers, GLB
//                                         BIN chunk; images decoded on threads
//   loadTriangles     stage1.zig:217-259  node order, primitive order; positions
//                                         by the node's global matrix, normals
//                                         by its 3x3 part then normalize (no
//                                         inverse transpose, as the reference)
//   loadCamera        stage1.zig:282-371  name lookup, first node carrying it
//   loadMaterials     stage1.zig:381-496  factor x linear texels, 1x1 dummies,
//                                         clamp/repeat ranges, MASK/BLEND alpha
//
// Where the reference is undefined or crashes (missing NORMAL/TEXCOORD_0
// reads undefined memory, missing indices/material hit `.?`), this loader
// defines the behaviour: zeros for missing attributes, sequential indices for
// non-indexed primitives, and an error for a primitive without material.
// zgltf's TRS composition and matrix product order are not recoverable
// offline (submodule empty): "parity unpinned" for node transforms that are
// not identity.  Images: PNG (png.cpp) and JPEG (jpeg.cpp) decoders.
#include <sys/stat.h>

#include <array>
#include <cmath>
#include <memory>
#include <new>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "json.h"
#include "png.h"
#include "zrt_internal.h"

using namespace zrt;
using json::Value;

struct zrt_gltf {
    std::vector<float> pos, nrm, uv;
    std::vector<uint32_t> mat;
    std::vector<zrt_material> materials;
    std::vector<float> texels;
    struct Cam {
        std::string name;
        bool perspective = true;
        float yfov = 0.8f;
        bool has_aspect = false;
        float aspect = 1.0f;
    };
    std::vector<Cam> cameras;
    std::vector<int> node_camera;          // camera index per node (-1)
    std::vector<std::array<float, 16>> node_global;
};

namespace {

bool read_file(const std::string& path, std::vector<uint8_t>* out) {
    struct stat sb;
    // a regular file only: a URI naming a directory opens, and its "size" is
    // LONG_MAX on some filesystems (found by tests/test_sanitize.py)
    if (stat(path.c_str(), &sb) != 0 || !S_ISREG(sb.st_mode)) return false;
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) return false;
    fseek(f, 0, SEEK_END);
    const long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    if (n < 0 || (uint64_t)n > (1ull << 34)) { fclose(f); return false; }
    out->resize((size_t)n);
    const size_t r = n ? fread(out->data(), 1, (size_t)n, f) : 0;
    fclose(f);
    return r == (size_t)n;
}

std::string dirname_of(const std::string& p) {
    const size_t k = p.find_last_of('/');
    return k == std::string::npos ? std::string(".") : p.substr(0, k);
}

std::string uri_decode(const std::string& s) {
    std::string o;
    for (size_t i = 0; i < s.size(); ++i) {
        if (s[i] == '%' && i + 2 < s.size()) {
            o.push_back((char)strtol(s.substr(i + 1, 2).c_str(), nullptr, 16));
            i += 2;
        } else {
            o.push_back(s[i]);
        }
    }
    return o;
}

bool base64(const std::string& s, std::vector<uint8_t>* out) {
    auto val = [](char c) -> int {
        if (c >= 'A' && c <= 'Z') return c - 'A';
        if (c >= 'a' && c <= 'z') return c - 'a' + 26;
        if (c >= '0' && c <= '9') return c - '0' + 52;
        if (c == '+') return 62;
        if (c == '/') return 63;
        return -1;
    };
    uint32_t acc = 0;
    int bits = 0;
    for (char c : s) {
        if (c == '=') break;
        const int v = val(c);
        if (v < 0) {
            if (c == '\n' || c == '\r' || c == ' ') continue;
            return false;
        }
        acc = (acc << 6) | (uint32_t)v;
        bits += 6;
        if (bits >= 8) { bits -= 8; out->push_back((uint8_t)(acc >> bits)); }
    }
    return true;
}

// uri -> bytes (data URI or file relative to the glTF's directory)
bool load_uri(const std::string& dir, const std::string& uri, std::vector<uint8_t>* out) {
    if (uri.compare(0, 5, "data:") == 0) {
        const size_t k = uri.find(";base64,");
        if (k == std::string::npos) return false;
        return base64(uri.substr(k + 8), out);
    }
    return read_file(dir + "/" + uri_decode(uri), out);
}

typedef std::array<float, 16> M4;   // column-major, m[col*4 + row]

M4 identity() { M4 m{}; m[0] = m[5] = m[10] = m[15] = 1.0f; return m; }
M4 mul(const M4& a, const M4& b) {
    M4 r{};
    for (int c = 0; c < 4; ++c)
        for (int rr = 0; rr < 4; ++rr) {
            float s = 0.0f;
            for (int k = 0; k < 4; ++k) s += a[k * 4 + rr] * b[c * 4 + k];
            r[c * 4 + rr] = s;
        }
    return r;
}
M4 local_transform(const Value& node) {
    if (const Value* m = node.get("matrix")) {
        M4 r = identity();
        if (m->type == Value::Array && m->size() == 16)
            for (int i = 0; i < 16; ++i) r[i] = (float)(*m)[i].num;
        return r;
    }
    float t[3] = {0, 0, 0}, q[4] = {0, 0, 0, 1}, s[3] = {1, 1, 1};
    if (const Value* v = node.get("translation")) for (int i = 0; i < 3 && i < (int)v->size(); ++i) t[i] = (float)(*v)[i].num;
    if (const Value* v = node.get("rotation")) for (int i = 0; i < 4 && i < (int)v->size(); ++i) q[i] = (float)(*v)[i].num;
    if (const Value* v = node.get("scale")) for (int i = 0; i < 3 && i < (int)v->size(); ++i) s[i] = (float)(*v)[i].num;
    const float x = q[0], y = q[1], z = q[2], w = q[3];
    M4 r{};
    r[0] = (1 - 2 * (y * y + z * z)) * s[0];
    r[1] = (2 * (x * y + w * z)) * s[0];
    r[2] = (2 * (x * z - w * y)) * s[0];
    r[4] = (2 * (x * y - w * z)) * s[1];
    r[5] = (1 - 2 * (x * x + z * z)) * s[1];
    r[6] = (2 * (y * z + w * x)) * s[1];
    r[8] = (2 * (x * z + w * y)) * s[2];
    r[9] = (2 * (y * z - w * x)) * s[2];
    r[10] = (1 - 2 * (x * x + y * y)) * s[2];
    r[12] = t[0]; r[13] = t[1]; r[14] = t[2]; r[15] = 1.0f;
    return r;
}

// Mat4.transformPosition / transformDirection (linalg.zig:262-277):
// col0*x + col1*y + col2*z (+ col3), vector adds left to right.
v3 col3(const M4& m, int c) { return mk(m[c * 4], m[c * 4 + 1], m[c * 4 + 2]); }
v3 xform_pos(const M4& m, v3 v) {
    return add(add(add(scale(col3(m, 0), v.x), scale(col3(m, 1), v.y)), scale(col3(m, 2), v.z)), col3(m, 3));
}
v3 xform_dir(const M4& m, v3 v) {
    return add(add(scale(col3(m, 0), v.x), scale(col3(m, 1), v.y)), scale(col3(m, 2), v.z));
}

struct Loader {
    Value doc;
    std::string dir;
    std::vector<std::vector<uint8_t>> buffers;
    std::vector<uint8_t> glb_bin;
    bool is_glb = false;

    struct Acc {
        const uint8_t* base = nullptr;
        size_t count = 0, stride = 0;
        int ctype = 0, ncomp = 0;
        bool normalized = false;
    };

    int accessor(int64_t idx, Acc* a) {
        const Value* accs = doc.get("accessors");
        if (!accs || idx < 0 || (size_t)idx >= accs->size()) return ZRT_ERR_PARSE;
        const Value& ac = (*accs)[(size_t)idx];
        if (ac.get("sparse")) return ZRT_ERR_UNSUPPORTED;
        const std::string type = ac.string("type", "");
        a->ncomp = type == "SCALAR" ? 1 : type == "VEC2" ? 2 : type == "VEC3" ? 3 : type == "VEC4" ? 4 : 0;
        a->ctype = (int)ac.integer("componentType", 0);
        const int64_t count = ac.integer("count", 0);
        a->normalized = ac.get("normalized") && ac.get("normalized")->b;
        int csz;
        switch (a->ctype) {
            case 5120: case 5121: csz = 1; break;
            case 5122: case 5123: csz = 2; break;
            case 5125: case 5126: csz = 4; break;
            default: return ZRT_ERR_PARSE;
        }
        const int64_t bv = ac.integer("bufferView", -1);
        if (bv < 0 || a->ncomp == 0) return ZRT_ERR_UNSUPPORTED;
        const Value* bvs = doc.get("bufferViews");
        if (!bvs || (size_t)bv >= bvs->size()) return ZRT_ERR_PARSE;
        const Value& v = (*bvs)[(size_t)bv];
        const int64_t b = v.integer("buffer", -1);
        if (b < 0 || (size_t)b >= buffers.size()) return ZRT_ERR_PARSE;
        // every size from the document checked before any arithmetic on it
        // (a hostile count/offset/stride must not wrap the bounds check)
        const int64_t o1 = v.integer("byteOffset", 0), o2 = ac.integer("byteOffset", 0);
        const int64_t st = v.integer("byteStride", 0);
        const uint64_t size = buffers[(size_t)b].size(), elem = (uint64_t)csz * a->ncomp;
        if (count < 0 || count > (1ll << 31) || o1 < 0 || o2 < 0 || st < 0 || st > 255) return ZRT_ERR_PARSE;
        if ((uint64_t)o1 > size || (uint64_t)o2 > size - (uint64_t)o1) return ZRT_ERR_PARSE;
        const uint64_t off = (uint64_t)o1 + (uint64_t)o2;
        a->count = (size_t)count;
        a->stride = st ? (size_t)st : (size_t)elem;
        if (st && (uint64_t)st < elem) return ZRT_ERR_PARSE;
        if (a->count) {
            if (size - off < elem) return ZRT_ERR_PARSE;
            if ((uint64_t)(a->count - 1) > (size - off - elem) / a->stride) return ZRT_ERR_PARSE;
        }
        a->base = buffers[(size_t)b].data() + off;
        return ZRT_OK;
    }
    static float comp_f(const Acc& a, size_t i, int c) {
        const uint8_t* p = a.base + i * a.stride;
        switch (a.ctype) {
            case 5126: { float f; memcpy(&f, p + 4 * c, 4); return f; }
            case 5121: return a.normalized ? p[c] / 255.0f : (float)p[c];
            case 5123: { uint16_t u; memcpy(&u, p + 2 * c, 2); return a.normalized ? u / 65535.0f : (float)u; }
            default: return 0.0f;
        }
    }
    static uint32_t index(const Acc& a, size_t i) {
        const uint8_t* p = a.base + i * a.stride;
        switch (a.ctype) {
            case 5121: return p[0];
            case 5123: { uint16_t u; memcpy(&u, p, 2); return u; }
            case 5125: { uint32_t u; memcpy(&u, p, 4); return u; }
            default: return 0;
        }
    }
};

int load_images(Loader& L, uint32_t nthreads, std::vector<Image8>* images) {
    const Value* imgs = L.doc.get("images");
    const size_t n = imgs ? imgs->size() : 0;
    images->assign(n, Image8());
    if (!n) return ZRT_OK;
    std::vector<int> rc(n, ZRT_OK);
    auto work = [&](size_t t, size_t nt) {   // stage1.zig:36-37 round-robin over threads
        for (size_t i = t; i < n; i += nt) {
            const Value& im = (*imgs)[i];
            std::vector<uint8_t> bytes;
            const uint8_t* data = nullptr;
            size_t len = 0;
            const int64_t bv = im.integer("bufferView", -1);
            if (bv >= 0) {
                const Value* bvs = L.doc.get("bufferViews");
                if (!bvs || (size_t)bv >= bvs->size()) { rc[i] = ZRT_ERR_PARSE; continue; }
                const Value& v = (*bvs)[(size_t)bv];
                const int64_t b = v.integer("buffer", -1);
                const size_t off = (size_t)v.integer("byteOffset", 0), bl = (size_t)v.integer("byteLength", 0);
                if (b < 0 || (size_t)b >= L.buffers.size() || off + bl > L.buffers[(size_t)b].size()) {
                    rc[i] = ZRT_ERR_PARSE;
                    continue;
                }
                data = L.buffers[(size_t)b].data() + off;
                len = bl;
            } else {
                if (!load_uri(L.dir, im.string("uri", ""), &bytes)) { rc[i] = ZRT_ERR_IO; continue; }
                data = bytes.data();
                len = bytes.size();
            }
            try {   // (a worker thread: nothing may escape it)
                rc[i] = (len >= 2 && data[0] == 0xFF && data[1] == 0xD8) ? jpeg_decode(data, len, &(*images)[i])
                                                                          : png_decode(data, len, &(*images)[i]);
            } catch (const std::bad_alloc&) {
                rc[i] = ZRT_ERR_OUT_OF_MEMORY;
            }
        }
    };
    const size_t nt = std::max<size_t>(1, std::min<size_t>(nthreads ? nthreads : host_threads(), n));
    std::vector<std::thread> th;
    for (size_t t = 1; t < nt; ++t) th.emplace_back(work, t, nt);
    work(0, nt);
    for (auto& x : th) x.join();
    for (int r : rc)
        if (r != ZRT_OK) return r;
    return ZRT_OK;
}

}  // namespace

static int gltf_load(const char* path, uint32_t num_threads, zrt_gltf** out);

// No exception crosses the C ABI: an allocation a hostile file provokes
// (sizes are validated against the data first) becomes an error code.
extern "C" int zrt_gltf_load(const char* path, uint32_t num_threads, zrt_gltf** out) {
    if (!path || !out) return ZRT_ERR_INVALID_ARG;
    *out = nullptr;
    try {
        return gltf_load(path, num_threads, out);
    } catch (const std::bad_alloc&) {
        return ZRT_ERR_OUT_OF_MEMORY;
    } catch (...) {
        return ZRT_ERR_PARSE;
    }
}

static int gltf_load(const char* path, uint32_t num_threads, zrt_gltf** out) {
    Loader L;
    L.dir = dirname_of(path);
    std::vector<uint8_t> file;
    if (!read_file(path, &file)) return ZRT_ERR_IO;
    const char* js = (const char*)file.data();
    size_t jn = file.size();
    if (file.size() >= 12 && memcmp(file.data(), "glTF", 4) == 0) {   // GLB container
        L.is_glb = true;
        size_t pos = 12;
        js = nullptr;
        while (pos + 8 <= file.size()) {
            uint32_t clen, ctype;
            memcpy(&clen, file.data() + pos, 4);
            memcpy(&ctype, file.data() + pos + 4, 4);
            if (clen > file.size() - pos - 8) return ZRT_ERR_PARSE;
            if (ctype == 0x4E4F534Au) { js = (const char*)file.data() + pos + 8; jn = clen; }
            else if (ctype == 0x004E4942u) L.glb_bin.assign(file.data() + pos + 8, file.data() + pos + 8 + clen);
            pos += 8 + ((clen + 3) & ~3u);
        }
        if (!js) return ZRT_ERR_PARSE;
    }
    if (!json::parse(js, jn, &L.doc) || L.doc.type != Value::Object) return ZRT_ERR_PARSE;

    // buffers (stage1.zig:86-95)
    if (const Value* bufs = L.doc.get("buffers")) {
        for (size_t i = 0; i < bufs->size(); ++i) {
            const Value& b = (*bufs)[i];
            std::vector<uint8_t> data;
            if (!b.get("uri")) {
                if (i != 0 || !L.is_glb) return ZRT_ERR_PARSE;
                data = L.glb_bin;
            } else if (!load_uri(L.dir, b.string("uri", ""), &data)) {
                return ZRT_ERR_IO;
            }
            L.buffers.push_back(std::move(data));
        }
    }
    std::vector<Image8> images;
    int rc = load_images(L, num_threads, &images);
    if (rc != ZRT_OK) return rc;

    zrt_gltf* g = new zrt_gltf();
    std::unique_ptr<zrt_gltf> guard(g);
    // node hierarchy -> global transforms (zgltf getGlobalTransform: parent * local)
    const Value* nodes = L.doc.get("nodes");
    const size_t nn = nodes ? nodes->size() : 0;
    std::vector<int> parent(nn, -1);
    for (size_t i = 0; i < nn; ++i)
        if (const Value* ch = (*nodes)[i].get("children"))
            for (size_t k = 0; k < ch->size(); ++k) {
                const int64_t c = (int64_t)(*ch)[k].num;
                if (c >= 0 && (size_t)c < nn) parent[(size_t)c] = (int)i;
            }
    g->node_global.resize(nn);
    g->node_camera.assign(nn, -1);
    for (size_t i = 0; i < nn; ++i) {
        M4 m = local_transform((*nodes)[i]);
        int p = parent[i];
        for (size_t guard_n = 0; p >= 0 && guard_n < nn; ++guard_n) {
            m = mul(local_transform((*nodes)[(size_t)p]), m);
            p = parent[(size_t)p];
        }
        g->node_global[i] = m;
        g->node_camera[i] = (int)(*nodes)[i].integer("camera", -1);
    }
    // triangles (stage1.zig:217-259)
    const Value* meshes = L.doc.get("meshes");
    for (size_t ni = 0; ni < nn; ++ni) {
        const int64_t mi = (*nodes)[ni].integer("mesh", -1);
        if (mi < 0) continue;
        if (!meshes || (size_t)mi >= meshes->size()) return ZRT_ERR_PARSE;
        const Value* prims = (*meshes)[(size_t)mi].get("primitives");
        if (!prims) continue;
        const M4& M = g->node_global[ni];
        for (size_t pi = 0; pi < prims->size(); ++pi) {
            const Value& pr = (*prims)[pi];
            if (pr.integer("mode", 4) != 4) return ZRT_ERR_UNSUPPORTED;
            const Value* attrs = pr.get("attributes");
            if (!attrs) return ZRT_ERR_PARSE;
            Loader::Acc ap, an, at, ai;
            if ((rc = L.accessor(attrs->integer("POSITION", -1), &ap)) != ZRT_OK) return rc;
            if (ap.ctype != 5126 || ap.ncomp != 3) return ZRT_ERR_UNSUPPORTED;
            const bool has_n = attrs->get("NORMAL") != nullptr, has_t = attrs->get("TEXCOORD_0") != nullptr;
            if (has_n && ((rc = L.accessor(attrs->integer("NORMAL", -1), &an)) != ZRT_OK)) return rc;
            if (has_n && (an.ctype != 5126 || an.ncomp != 3)) return ZRT_ERR_UNSUPPORTED;
            if (has_t && ((rc = L.accessor(attrs->integer("TEXCOORD_0", -1), &at)) != ZRT_OK)) return rc;
            if (has_t && (at.ncomp != 2 || !(at.ctype == 5126 || at.ctype == 5121 || at.ctype == 5123)))
                return ZRT_ERR_UNSUPPORTED;
            const bool indexed = pr.get("indices") != nullptr;
            if (indexed && ((rc = L.accessor(pr.integer("indices", -1), &ai)) != ZRT_OK)) return rc;
            if (indexed && (ai.ncomp != 1 || !(ai.ctype == 5121 || ai.ctype == 5123 || ai.ctype == 5125)))
                return ZRT_ERR_PARSE;
            const int64_t mat = pr.integer("material", -1);
            if (mat < 0) return ZRT_ERR_UNSUPPORTED;   // reference: primitive.material.? (stage1.zig:239)
            const size_t nidx = indexed ? ai.count : ap.count;
            for (size_t t = 0; t + 3 <= nidx; t += 3) {
                for (int k = 0; k < 3; ++k) {
                    const uint32_t vi = indexed ? Loader::index(ai, t + k) : (uint32_t)(t + k);
                    if (vi >= ap.count || (has_n && vi >= an.count) || (has_t && vi >= at.count))
                        return ZRT_ERR_PARSE;
                    const v3 p = xform_pos(M, mk(Loader::comp_f(ap, vi, 0), Loader::comp_f(ap, vi, 1),
                                                 Loader::comp_f(ap, vi, 2)));
                    const v3 nv = has_n ? normalize(xform_dir(M, mk(Loader::comp_f(an, vi, 0),
                                                                     Loader::comp_f(an, vi, 1),
                                                                     Loader::comp_f(an, vi, 2))))
                                        : mk(0, 0, 0);
                    g->pos.insert(g->pos.end(), {p.x, p.y, p.z});
                    g->nrm.insert(g->nrm.end(), {nv.x, nv.y, nv.z});
                    g->uv.push_back(has_t ? Loader::comp_f(at, vi, 0) : 0.0f);
                    g->uv.push_back(has_t ? Loader::comp_f(at, vi, 1) : 0.0f);
                }
                g->mat.push_back((uint32_t)mat);
            }
        }
    }
    // materials (stage1.zig:381-496)
    const Value* mats = L.doc.get("materials");
    const Value* texs = L.doc.get("textures");
    const Value* samplers = L.doc.get("samplers");
    auto push = [&](const float* src, size_t n) {
        const uint64_t off = g->texels.size();
        g->texels.insert(g->texels.end(), src, src + n);
        return off;
    };
    // texture index -> (image, clamp ranges) (stage1.zig:381-409)
    auto tex_info = [&](int64_t ti, int* img, zrt_texture* t) -> int {
        if (!texs || ti < 0 || (size_t)ti >= texs->size()) return ZRT_ERR_PARSE;
        const Value& tx = (*texs)[(size_t)ti];
        const int64_t src = tx.integer("source", -1);
        if (src < 0 || (size_t)src >= images.size()) return ZRT_ERR_UNSUPPORTED;
        *img = (int)src;
        const Image8& im = images[(size_t)src];
        t->w = im.w;
        t->h = im.h;
        t->u_min = INT32_MIN; t->u_max = INT32_MAX; t->v_min = INT32_MIN; t->v_max = INT32_MAX;
        const int64_t si = tx.integer("sampler", -1);
        if (si >= 0 && samplers && (size_t)si < samplers->size()) {
            const Value& s = (*samplers)[(size_t)si];
            if (s.integer("wrapS", 10497) == 33071) { t->u_min = 0; t->u_max = im.w - 1; }
            if (s.integer("wrapT", 10497) == 33071) { t->v_min = 0; t->v_max = im.h - 1; }
        }
        return ZRT_OK;
    };
    std::vector<std::vector<float>> linear(images.size());
    for (size_t i = 0; i < images.size(); ++i) rgba8_to_linear(images[i], &linear[i]);
    const size_t nmat = mats ? mats->size() : 0;
    g->materials.resize(nmat);
    for (size_t m = 0; m < nmat; ++m) {
        const Value& mv = (*mats)[m];
        const Value* pbr = mv.get("pbrMetallicRoughness");
        float bcf[4] = {1, 1, 1, 1}, ef[3] = {0, 0, 0};
        if (pbr)
            if (const Value* f = pbr->get("baseColorFactor"))
                for (int k = 0; k < 4 && k < (int)f->size(); ++k) bcf[k] = (float)(*f)[k].num;
        if (const Value* f = mv.get("emissiveFactor"))
            for (int k = 0; k < 3 && k < (int)f->size(); ++k) ef[k] = (float)(*f)[k].num;
        // loadColorTexture
        auto color = [&](const Value* info, const float* factor, zrt_texture* t) -> int {
            if (!info) {
                t->offset = push(factor, 3);
                t->w = t->h = 1;
                t->u_min = t->u_max = t->v_min = t->v_max = 0;
                return ZRT_OK;
            }
            int img;
            const int r = tex_info(info->integer("index", -1), &img, t);
            if (r != ZRT_OK) return r;
            const std::vector<float>& lin = linear[(size_t)img];
            std::vector<float> rgb((size_t)t->w * t->h * 3);
            for (size_t i = 0; i < (size_t)t->w * t->h; ++i)
                for (int k = 0; k < 3; ++k) rgb[3 * i + k] = lin[4 * i + k] * factor[k];
            t->offset = push(rgb.data(), rgb.size());
            return ZRT_OK;
        };
        const Value* bct = pbr ? pbr->get("baseColorTexture") : nullptr;
        if ((rc = color(bct, bcf, &g->materials[m].base_color)) != ZRT_OK) return rc;
        if ((rc = color(mv.get("emissiveTexture"), ef, &g->materials[m].emissive)) != ZRT_OK) return rc;
        // loadTransparencyTexture
        zrt_texture& tt = g->materials[m].transparency;
        const std::string mode = mv.string("alphaMode", "OPAQUE");
        bool done = false;
        if (mode != "OPAQUE" && bct) {
            int img;
            zrt_texture t{};
            if ((rc = tex_info(bct->integer("index", -1), &img, &t)) != ZRT_OK) return rc;
            const Image8& im = images[(size_t)img];
            if (im.actual_c == 4 || im.actual_c == 2) {
                const float cutoff = (float)mv.number("alphaCutoff", 0.5);
                const std::vector<float>& lin = linear[(size_t)img];
                std::vector<float> a((size_t)t.w * t.h);
                for (size_t i = 0; i < a.size(); ++i) {
                    const float al = lin[4 * i + 3];
                    a[i] = mode == "MASK" ? (al > cutoff ? 1.0f : 0.0f) : al;
                }
                t.offset = push(a.data(), a.size());
                tt = t;
                done = true;
            }
        }
        if (!done) {
            const float one = 1.0f;
            tt.offset = push(&one, 1);
            tt.w = tt.h = 1;
            tt.u_min = tt.u_max = tt.v_min = tt.v_max = 0;
        }
    }
    for (uint32_t m : g->mat)
        if (m >= nmat) return ZRT_ERR_PARSE;
    // cameras
    if (const Value* cams = L.doc.get("cameras"))
        for (size_t i = 0; i < cams->size(); ++i) {
            const Value& c = (*cams)[i];
            zrt_gltf::Cam cam;
            cam.name = c.string("name", "");
            cam.perspective = c.string("type", "perspective") == "perspective";
            if (const Value* p = c.get("perspective")) {
                cam.yfov = (float)p->number("yfov", 0.8);
                cam.has_aspect = p->get("aspectRatio") != nullptr;
                cam.aspect = (float)p->number("aspectRatio", 1.0);
            } else {
                cam.perspective = false;
            }
            g->cameras.push_back(cam);
        }
    *out = guard.release();
    return ZRT_OK;
}

extern "C" int zrt_gltf_soup(const zrt_gltf* g, const float** positions, const float** normals,
                             const float** texcoords, const uint32_t** material, uint32_t* n) {
    if (!g || !positions || !normals || !texcoords || !material || !n) return ZRT_ERR_INVALID_ARG;
    *positions = g->pos.data();
    *normals = g->nrm.data();
    *texcoords = g->uv.data();
    *material = g->mat.data();
    *n = (uint32_t)g->mat.size();
    return ZRT_OK;
}

extern "C" int zrt_gltf_materials(const zrt_gltf* g, zrt_scene* s) {
    if (!g || !s) return ZRT_ERR_INVALID_ARG;
    s->num_materials = (uint32_t)g->materials.size();
    s->materials = g->materials.data();
    s->texels = g->texels.data();
    s->num_texel_floats = g->texels.size();
    return ZRT_OK;
}

// stage1.zig:282-371 (findCameraIndex, findCameraNode, loadCamera)
extern "C" int zrt_gltf_camera(const zrt_gltf* g, const char* name, int32_t width, int32_t height,
                               zrt_camera* out) {
    if (!g || !out) return ZRT_ERR_INVALID_ARG;
    if (g->cameras.empty()) return ZRT_ERR_NOT_FOUND;                 // NoCamerasAtAll
    int idx = 0;
    if (name) {
        idx = -1;
        for (size_t i = 0; i < g->cameras.size(); ++i)
            if (g->cameras[i].name == name) { idx = (int)i; break; }
        if (idx < 0) return ZRT_ERR_NOT_FOUND;                        // CameraNotFound
    }
    int node = -1;
    for (size_t i = 0; i < g->node_camera.size(); ++i)
        if (g->node_camera[i] == idx) { node = (int)i; break; }
    if (node < 0) return ZRT_ERR_NOT_FOUND;                           // CameraNodeNotFound
    const zrt_gltf::Cam& c = g->cameras[(size_t)idx];
    if (!c.perspective) return ZRT_ERR_UNSUPPORTED;                   // OnlyPerspectiveCamerasSupported
    return zrt_camera_from_matrix(g->node_global[(size_t)node].data(), c.yfov, c.has_aspect ? 1 : 0,
                                  c.aspect, width, height, out);
}

extern "C" void zrt_gltf_free(zrt_gltf* g) { delete g; }
