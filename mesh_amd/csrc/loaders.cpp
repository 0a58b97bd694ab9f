// Native mesh loaders feeding the search path: OBJ (replaces
// mesh/src/py_loadobj.cpp, the `psbody.mesh.serialization.loadobj` extension) and PLY (replaces
// mesh/src/plyutils.c `plyutils.read` over rply.c).  Host code: the file is memory-mapped and parsed in
// one pass straight into the arrays the caller copies out (no per-line string copies, no
// istringstream); the outputs are the reference's, value for value.
//
// OBJ semantics (py_loadobj.cpp:104-190), line by line, in the reference's order of tests:
//   "mtllib"   -> mtl_path = the rest of the line after the 6 letters (leading space kept)
//   "g"        -> current group = line from column 2; a new name starts an empty group
//   "vt" / "vn" / "f" / "v" (else-if chain, in this order), "#landmark" -> the next "v" is a landmark
//   numbers: whitespace-separated tokens parsed as by `istream >> double` until the first token that is
//   not a number (strtod rounding; "inf"/"nan" stop the line as num_get does)
//   "f": tokens "v", "v/vt", "v/vt/vn", "v//vn"; each '/'-separated element, if non-empty, is atoi'd
//   into f / ft / fn by its position; polygons are fan-triangulated (0, i, i+1); indices are 1-based
//   and stored minus one as uint32 (so 0 or negative indices wrap, as in the reference)
//   faces of a named group are appended to it (face index in f)
//   vt rows have the width of the LAST vt line (3 if there is none)
// Deviations (defects of the reference, SURVEY App. B style): a "g" line shorter than 2 characters
// (std::out_of_range there) names group ""; a vt line with no numbers makes vt empty instead of a
// division by zero; v / vt / vn values beyond a whole row are dropped instead of overrunning the array.
//
// PLY semantics (plyutils.c:64-139, rply.c): magic "ply\n" (else "Failed to open PLY file."), header
// "format ascii|binary_little_endian|binary_big_endian 1.0", "comment"/"obj_info" lines, elements with
// scalar properties of the rply types and list properties; vertex x, y, z (+ red, green, blue if any of
// them exists, + nx, ny, nz likewise) and face "vertex_indices" (or "vertex_index" when the former has no
// faces): items 0..2 of each list (further items are ignored, as face_cb does).  All values are
// converted to double (ascii: strtol / strtod with rply's range checks; binary: the raw value).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/meshsearch.h"

namespace msh {
void set_error(const char* fmt, ...);
}

namespace {

struct Mapped {
    const char* p = nullptr;
    size_t n = 0;
    int fd = -1;
    bool open(const char* path) {
        fd = ::open(path, O_RDONLY);
        if (fd < 0) return false;
        struct stat st;
        if (fstat(fd, &st) != 0 || !S_ISREG(st.st_mode)) return false;
        n = (size_t)st.st_size;
        if (n == 0) {
            p = "";
            return true;
        }
        void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
        if (m == MAP_FAILED) return false;
        p = static_cast<const char*>(m);
        madvise(m, n, MADV_SEQUENTIAL);
        return true;
    }
    ~Mapped() {
        if (p && n) munmap(const_cast<char*>(p), n);
        if (fd >= 0) ::close(fd);
    }
};

inline bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; }

// istream >> double over [s, e): tokens until the first non-number.  strtod needs a terminated string:
// tokens are copied into a small buffer (numbers are short).
void parse_doubles(const char* s, const char* e, std::vector<double>& out) {
    char buf[128];
    while (true) {
        while (s < e && is_ws(*s)) ++s;
        if (s >= e) return;
        const char* t = s;
        while (t < e && !is_ws(*t)) ++t;
        const size_t len = (size_t)(t - s) < sizeof(buf) - 1 ? (size_t)(t - s) : sizeof(buf) - 1;
        std::memcpy(buf, s, len);
        buf[len] = 0;
        // num_get accepts [+-]digits[.digits][e[+-]digits]; it rejects inf / nan and hex
        const char* b = buf + ((buf[0] == '+' || buf[0] == '-') ? 1 : 0);
        if (!((*b >= '0' && *b <= '9') || *b == '.')) return;
        if (b[0] == '0' && (b[1] == 'x' || b[1] == 'X')) {
            out.push_back(0.0);  // "0x..." reads as 0, then the stream fails at 'x'
            return;
        }
        char* end = nullptr;
        const double v = strtod(buf, &end);
        if (end == buf) return;
        out.push_back(v);
        if ((size_t)(end - buf) != len) return;  // "1.5abc": 1.5 then the next extraction fails
        s = t;
    }
}

}  // namespace

struct msh_obj {
    std::vector<double> v, vt, vn;
    std::vector<uint32_t> f, ft, fn;
    size_t len_vt = 3;
    std::string mtl_path;
    std::map<std::string, std::vector<uint32_t>> segm;
    std::map<std::string, uint32_t> landm;
};

struct msh_ply {
    std::vector<double> v, tri, color, normals;
    size_t nv = 0, nf = 0;
    bool has_color = false, has_normals = false;
};

using msh::set_error;

namespace {

// Runs a loader body so that no C++ exception crosses the extern "C" boundary: an allocation failure
// becomes MSH_ENOMEM, anything else MSH_EINVAL, each with a message (the Python shim raises the module's
// error for both).
template <class F>
int guarded(const char* what, F&& body) {
    try {
        return body();
    } catch (const std::bad_alloc&) {
        set_error("%s: out of memory", what);
        return MSH_ENOMEM;
    } catch (const std::length_error&) {
        set_error("%s: sizes too large", what);
        return MSH_ENOMEM;
    } catch (const std::exception& e) {
        set_error("%s: %s", what, e.what());
        return MSH_EINVAL;
    } catch (...) {
        set_error("%s: unknown error", what);
        return MSH_EINVAL;
    }
}

int obj_load(const char* path, msh_obj** out) {
    Mapped m;
    if (!m.open(path)) {
        set_error("Could not load file");
        return MSH_EINVAL;
    }
    std::unique_ptr<msh_obj> o(new msh_obj());
    o->v.reserve(30000);
    o->f.reserve(100000);
    bool next_v_is_land = false;
    std::string land_name, curr;
    std::vector<uint32_t> lf, lt, ln;
    const char* p = m.p;
    const char* end = m.p + m.n;
    while (p < end) {
        const char* nl = static_cast<const char*>(memchr(p, '\n', (size_t)(end - p)));
        const char* le = nl ? nl : end;  // line [p, le), as getline returns it
        const size_t L = (size_t)(le - p);
        auto starts = [&](const char* pre, size_t k) { return L >= k && std::memcmp(p, pre, k) == 0; };
        if (starts("mtllib", 6)) o->mtl_path.assign(p + 6, le);
        if (starts("g", 1)) {
            curr = L >= 2 ? std::string(p + 2, le) : std::string();
            o->segm.emplace(curr, std::vector<uint32_t>());
        }
        if (starts("vt", 2)) {
            const size_t before = o->vt.size();
            parse_doubles(p + 2, le, o->vt);
            o->len_vt = o->vt.size() - before;
        } else if (starts("vn", 2)) {
            parse_doubles(p + 2, le, o->vn);
        } else if (starts("f", 1)) {
            lf.clear();
            lt.clear();
            ln.clear();
            const char* s = p + 1;
            while (true) {
                while (s < le && is_ws(*s)) ++s;
                if (s >= le) break;
                const char* t = s;
                while (t < le && !is_ws(*t)) ++t;
                // elements of the token split at '/', empty ones skipped but counted
                int counter = 0;
                const char* a = s;
                while (a <= t) {
                    const char* b = a;
                    while (b < t && *b != '/') ++b;
                    if (b > a) {
                        const int x = atoi(std::string(a, b).c_str());
                        if (counter == 0) lf.push_back((uint32_t)x);
                        if (counter == 1) lt.push_back((uint32_t)x);
                        if (counter == 2) ln.push_back((uint32_t)x);
                    }
                    ++counter;
                    if (b >= t) break;
                    a = b + 1;
                    if (a == t) break;  // a trailing '/' ends the token (getline yields no empty tail)
                }
                s = t;
            }
            for (size_t i = 1; i + 1 < lf.size(); ++i) {
                o->f.push_back(lf[0] - 1u);
                o->f.push_back(lf[i] - 1u);
                o->f.push_back(lf[i + 1] - 1u);
                if (!curr.empty()) o->segm[curr].push_back((uint32_t)(o->f.size() / 3 - 1));
            }
            for (size_t i = 1; i + 1 < lt.size(); ++i) {
                o->ft.push_back(lt[0] - 1u);
                o->ft.push_back(lt[i] - 1u);
                o->ft.push_back(lt[i + 1] - 1u);
            }
            for (size_t i = 1; i + 1 < ln.size(); ++i) {
                o->fn.push_back(ln[0] - 1u);
                o->fn.push_back(ln[i] - 1u);
                o->fn.push_back(ln[i + 1] - 1u);
            }
        } else if (starts("v", 1)) {
            parse_doubles(p + 1, le, o->v);
            if (next_v_is_land) {
                next_v_is_land = false;
                o->landm[land_name] = (uint32_t)(o->v.size() / 3 - 1);
            }
        } else if (starts("#landmark", 9)) {
            next_v_is_land = true;
            land_name = L >= 10 ? std::string(p + 10, le) : std::string();
        }
        p = nl ? nl + 1 : end;
    }
    *out = o.release();
    return MSH_OK;
}

}  // namespace

extern "C" {

int msh_obj_load(const char* path, msh_obj** out) {
    if (!path || !out) {
        set_error("msh_obj_load: null argument");
        return MSH_EINVAL;
    }
    *out = nullptr;
    return guarded("msh_obj_load", [&] { return obj_load(path, out); });
}

int msh_obj_sizes(const msh_obj* o, uint64_t* s) {
    if (!o || !s) {
        set_error("msh_obj_sizes: null argument");
        return MSH_EINVAL;
    }
    s[0] = o->v.size() / 3;
    s[1] = o->len_vt ? o->vt.size() / o->len_vt : 0;
    s[2] = o->len_vt;
    s[3] = o->vn.size() / 3;
    s[4] = o->f.size() / 3;
    s[5] = o->ft.size() / 3;
    s[6] = o->fn.size() / 3;
    s[7] = o->segm.size();
    s[8] = o->landm.size();
    return MSH_OK;
}

int msh_obj_arrays(const msh_obj* o, double* v, double* vt, double* vn, uint32_t* f, uint32_t* ft, uint32_t* fn) {
    if (!o) {
        set_error("msh_obj_arrays: null argument");
        return MSH_EINVAL;
    }
    uint64_t s[9];
    msh_obj_sizes(o, s);
    // an empty array has no storage (data() may be null): nothing to copy (memcpy's arguments must not be null,
    // even for 0 bytes; UBSan, scripts/asan_check.sh)
    auto put = [](void* dst, const void* src, size_t bytes) {
        if (dst && bytes) std::memcpy(dst, src, bytes);
    };
    put(v, o->v.data(), s[0] * 3 * sizeof(double));
    put(vt, o->vt.data(), s[1] * s[2] * sizeof(double));
    put(vn, o->vn.data(), s[3] * 3 * sizeof(double));
    put(f, o->f.data(), s[4] * 3 * sizeof(uint32_t));
    put(ft, o->ft.data(), s[5] * 3 * sizeof(uint32_t));
    put(fn, o->fn.data(), s[6] * 3 * sizeof(uint32_t));
    return MSH_OK;
}

const char* msh_obj_mtl_path(const msh_obj* o) { return o ? o->mtl_path.c_str() : ""; }

int msh_obj_group(const msh_obj* o, size_t k, const char** name, uint64_t* n, const uint32_t** faces) {
    if (!o || !name || !n || !faces || k >= o->segm.size()) {
        set_error("msh_obj_group: bad argument");
        return MSH_EINVAL;
    }
    auto it = o->segm.begin();
    std::advance(it, (long)k);
    *name = it->first.c_str();
    *n = it->second.size();
    *faces = it->second.data();
    return MSH_OK;
}

int msh_obj_landmark(const msh_obj* o, size_t k, const char** name, uint32_t* vertex) {
    if (!o || !name || !vertex || k >= o->landm.size()) {
        set_error("msh_obj_landmark: bad argument");
        return MSH_EINVAL;
    }
    auto it = o->landm.begin();
    std::advance(it, (long)k);
    *name = it->first.c_str();
    *vertex = it->second;
    return MSH_OK;
}

void msh_obj_free(msh_obj* o) { delete o; }

}  // extern "C"

// ---------------------------------------------------------------- PLY
namespace {

enum PType { kI8, kU8, kI16, kU16, kI32, kU32, kF32, kF64, kBad };

PType ptype(const std::string& s) {
    static const std::map<std::string, PType> t = {
        {"int8", kI8},   {"char", kI8},    {"uint8", kU8},  {"uchar", kU8},  {"int16", kI16},   {"short", kI16},
        {"uint16", kU16}, {"ushort", kU16}, {"int32", kI32}, {"int", kI32},   {"uint32", kU32},  {"uint", kU32},
        {"float32", kF32}, {"float", kF32}, {"float64", kF64}, {"double", kF64}};
    auto it = t.find(s);
    return it == t.end() ? kBad : it->second;
}
size_t psize(PType t) {
    switch (t) {
        case kI8: case kU8: return 1;
        case kI16: case kU16: return 2;
        case kI32: case kU32: case kF32: return 4;
        case kF64: return 8;
        default: return 0;
    }
}

struct Prop {
    std::string name;
    bool list = false;
    PType count = kBad, item = kBad;
};
struct Elem {
    std::string name;
    long n = 0;
    std::vector<Prop> props;
};

struct Reader {
    const char* p;
    const char* e;
    int mode;  // 0 ascii, 1 binary little endian, 2 binary big endian
    bool ok = true;
    // ascii: next whitespace-separated word
    bool word(std::string& w) {
        while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
        if (p >= e) return false;
        const char* s = p;
        while (p < e && !(*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
        w.assign(s, p);
        return true;
    }
    double value(PType t) {
        if (mode == 0) {
            std::string w;
            if (!word(w)) { ok = false; return 0.0; }
            // rply.c:1320-1382: strtol / strtod of the word, the whole word consumed, range-checked
            char* end = nullptr;
            double v;
            if (t == kF32 || t == kF64) v = strtod(w.c_str(), &end);
            else v = (double)strtol(w.c_str(), &end, 10);
            if (end == w.c_str() || *end) ok = false;
            static const double lim[8][2] = {{-128, 127}, {0, 255}, {-32768, 32767}, {0, 65535},
                                             {-2147483648.0, 2147483647.0}, {0, 4294967295.0},
                                             {-3.4028234663852886e38, 3.4028234663852886e38}, {-INFINITY, INFINITY}};
            if (v < lim[t][0] || v > lim[t][1]) ok = false;
            return v;
        }
        const size_t n = psize(t);
        if ((size_t)(e - p) < n) { ok = false; return 0.0; }
        unsigned char b[8];
        std::memcpy(b, p, n);
        p += n;
        if (mode == 2)
            for (size_t i = 0; i < n / 2; ++i) std::swap(b[i], b[n - 1 - i]);
        switch (t) {
            case kI8: { int8_t x; std::memcpy(&x, b, 1); return x; }
            case kU8: { uint8_t x; std::memcpy(&x, b, 1); return x; }
            case kI16: { int16_t x; std::memcpy(&x, b, 2); return x; }
            case kU16: { uint16_t x; std::memcpy(&x, b, 2); return x; }
            case kI32: { int32_t x; std::memcpy(&x, b, 4); return x; }
            case kU32: { uint32_t x; std::memcpy(&x, b, 4); return x; }
            case kF32: { float x; std::memcpy(&x, b, 4); return x; }
            case kF64: { double x; std::memcpy(&x, b, 8); return x; }
            default: ok = false; return 0.0;
        }
    }
};

// Fewest bytes one instance of `el` can occupy in the body (binary: the scalar sizes plus each list's
// count; ascii: one character and one separator per value, a list at least its count), never below 1, so
// an element count that the bytes after end_header cannot hold is refused before anything is allocated.
size_t min_elem_bytes(const Elem& el, int mode) {
    size_t b = 0;
    for (const auto& pr : el.props) b += mode == 0 ? 2 : psize(pr.list ? pr.count : pr.item);
    return b ? b : 1;
}

int ply_load(const char* path, msh_ply** out) {
    Mapped m;
    if (!m.open(path) || m.n < 4 || std::memcmp(m.p, "ply\n", 4) != 0) {
        set_error("Failed to open PLY file.");
        return MSH_EINVAL;
    }
    // ---- header: lines up to "end_header"
    const char* p = m.p + 4;
    const char* end = m.p + m.n;
    int mode = -1;
    std::vector<Elem> elems;
    bool header_ok = false;
    while (p < end) {
        const char* nl = static_cast<const char*>(memchr(p, '\n', (size_t)(end - p)));
        if (!nl) break;
        std::string line(p, nl);
        p = nl + 1;
        std::vector<std::string> w;
        {
            size_t i = 0;
            while (i < line.size()) {
                while (i < line.size() && (line[i] == ' ' || line[i] == '\t' || line[i] == '\r')) ++i;
                size_t j = i;
                while (j < line.size() && !(line[j] == ' ' || line[j] == '\t' || line[j] == '\r')) ++j;
                if (j > i) w.emplace_back(line.substr(i, j - i));
                i = j;
            }
        }
        if (w.empty()) continue;
        if (w[0] == "end_header") { header_ok = true; break; }
        if (w[0] == "comment" || w[0] == "obj_info") continue;
        if (w[0] == "format" && w.size() >= 3 && w[2] == "1.0") {
            mode = w[1] == "ascii" ? 0 : w[1] == "binary_little_endian" ? 1 : w[1] == "binary_big_endian" ? 2 : -1;
            if (mode < 0) break;
        } else if (w[0] == "element" && w.size() == 3) {
            Elem el;
            el.name = w[1];
            char* e = nullptr;
            errno = 0;
            el.n = strtol(w[2].c_str(), &e, 10);
            if (e == w[2].c_str() || *e || errno == ERANGE || el.n < 0) break;  // not a count: bad header
            elems.push_back(el);
        } else if (w[0] == "property" && !elems.empty()) {
            Prop pr;
            if (w.size() == 5 && w[1] == "list") {
                pr.list = true;
                pr.count = ptype(w[2]);
                pr.item = ptype(w[3]);
                pr.name = w[4];
                if (pr.count == kBad || pr.item == kBad) break;
            } else if (w.size() == 3) {
                pr.item = ptype(w[1]);
                pr.name = w[2];
                if (pr.item == kBad) break;
            } else {
                break;
            }
            elems.back().props.push_back(pr);
        } else {
            break;
        }
    }
    if (!header_ok || mode < 0) {
        set_error("plyread_mex: Bad raw header.");
        return MSH_EINVAL;
    }
    {
        const size_t left = (size_t)(end - p) + (mode == 0 ? 1 : 0);  // ascii: the last value needs no separator
        size_t need = 0;
        for (const auto& el : elems) {
            const size_t mb = min_elem_bytes(el, mode);
            if ((size_t)el.n > left / mb || need > left - (size_t)el.n * mb) {
                set_error("Read failed. %s: element '%s' count %ld exceeds the file", path, el.name.c_str(), el.n);
                return MSH_EINVAL;
            }
            need += (size_t)el.n * mb;
        }
    }
    std::unique_ptr<msh_ply> o(new msh_ply());
    // which vertex properties exist (plyutils.c has_color / has_normals)
    auto find = [&](const std::string& e) -> Elem* {
        for (auto& x : elems)
            if (x.name == e) return &x;
        return nullptr;
    };
    Elem* ve = find("vertex");
    Elem* fe = find("face");
    if (ve)
        for (auto& pr : ve->props) {
            if (pr.name == "red" || pr.name == "green" || pr.name == "blue") o->has_color = true;
            if (pr.name == "nx" || pr.name == "ny" || pr.name == "nz") o->has_normals = true;
        }
    o->nv = ve ? (size_t)ve->n : 0;
    std::string face_prop = "vertex_indices";
    bool have_fprop = false;
    if (fe)
        for (auto& pr : fe->props)
            if (pr.name == "vertex_indices") have_fprop = true;
    if (!have_fprop || !fe || fe->n == 0) {
        face_prop = "vertex_index";
        have_fprop = false;
        if (fe)
            for (auto& pr : fe->props)
                if (pr.name == "vertex_index") have_fprop = true;
    }
    o->nf = (fe && have_fprop) ? (size_t)fe->n : 0;
    o->v.assign(3 * o->nv, NAN);
    o->tri.assign(3 * o->nf, NAN);
    if (o->has_color) o->color.assign(3 * o->nv, NAN);
    if (o->has_normals) o->normals.assign(3 * o->nv, NAN);
    // ---- body
    Reader r{p, end, mode};
    for (auto& el : elems) {
        const bool isv = &el == ve, isf = &el == fe;
        for (long i = 0; i < el.n && r.ok; ++i) {
            for (auto& pr : el.props) {
                if (!pr.list) {
                    const double x = r.value(pr.item);
                    if (!r.ok) break;
                    if (isv) {
                        const char* n = pr.name.c_str();
                        const size_t b = 3 * (size_t)i;
                        if (!strcmp(n, "x")) o->v[b] = x;
                        else if (!strcmp(n, "y")) o->v[b + 1] = x;
                        else if (!strcmp(n, "z")) o->v[b + 2] = x;
                        else if (o->has_color && !strcmp(n, "red")) o->color[b] = x;
                        else if (o->has_color && !strcmp(n, "green")) o->color[b + 1] = x;
                        else if (o->has_color && !strcmp(n, "blue")) o->color[b + 2] = x;
                        else if (o->has_normals && !strcmp(n, "nx")) o->normals[b] = x;
                        else if (o->has_normals && !strcmp(n, "ny")) o->normals[b + 1] = x;
                        else if (o->has_normals && !strcmp(n, "nz")) o->normals[b + 2] = x;
                    }
                } else {
                    const double cnt = r.value(pr.count);
                    if (!r.ok || cnt < 0) { r.ok = false; break; }
                    const long c = (long)cnt;
                    for (long k = 0; k < c; ++k) {
                        const double x = r.value(pr.item);
                        if (!r.ok) break;
                        if (isf && pr.name == face_prop && k < 3) o->tri[3 * (size_t)i + (size_t)k] = x;
                    }
                }
            }
        }
        if (!r.ok) break;
    }
    if (!r.ok) {
        set_error("Read failed. %s", path);
        return MSH_EINVAL;
    }
    *out = o.release();
    return MSH_OK;
}

}  // namespace

extern "C" {

int msh_ply_load(const char* path, msh_ply** out) {
    if (!path || !out) {
        set_error("msh_ply_load: null argument");
        return MSH_EINVAL;
    }
    *out = nullptr;
    return guarded("msh_ply_load", [&] { return ply_load(path, out); });
}

int msh_ply_sizes(const msh_ply* o, uint64_t* s) {
    if (!o || !s) {
        set_error("msh_ply_sizes: null argument");
        return MSH_EINVAL;
    }
    s[0] = o->nv;
    s[1] = o->nf;
    s[2] = o->has_color ? 1 : 0;
    s[3] = o->has_normals ? 1 : 0;
    return MSH_OK;
}

int msh_ply_arrays(const msh_ply* o, double* v, double* tri, double* color, double* normals) {
    if (!o) {
        set_error("msh_ply_arrays: null argument");
        return MSH_EINVAL;
    }
    auto put = [](void* dst, const std::vector<double>& src) {  // empty: no storage, nothing to copy
        if (dst && !src.empty()) std::memcpy(dst, src.data(), src.size() * sizeof(double));
    };
    put(v, o->v);
    put(tri, o->tri);
    if (o->has_color) put(color, o->color);
    if (o->has_normals) put(normals, o->normals);
    return MSH_OK;
}

void msh_ply_free(msh_ply* o) { delete o; }

}  // extern "C"
