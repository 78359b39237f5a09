// GGUF reader/writer (see gguf.h).
#include "gguf.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cmath>
#include <cstring>

#include "common.h"

namespace mio {

size_t ggml_type_block_elems(uint32_t t) {
    switch (t) {
        case GGML_Q4_0:
        case GGML_Q5_0:
        case GGML_Q8_0: return 32;
        case GGML_Q4_K:
        case GGML_Q6_K:
        case GGML_Q8_K: return 256;
        default: return 1;
    }
}

size_t ggml_type_block_bytes(uint32_t t) {
    switch (t) {
        case GGML_F32: return 4;
        case GGML_F16: return 2;
        case GGML_BF16: return 2;
        case GGML_I8: return 1;
        case GGML_I16: return 2;
        case GGML_I32: return 4;
        case GGML_Q4_0: return 18;
        case GGML_Q5_0: return 22;
        case GGML_Q8_0: return 34;
        case GGML_Q4_K: return 144;
        case GGML_Q6_K: return 210;
        case GGML_Q8_K: return 292;
        default: return 0;
    }
}

size_t ggml_row_bytes(uint32_t t, int64_t n) {
    const size_t be = ggml_type_block_elems(t), bb = ggml_type_block_bytes(t);
    if (!bb || n % (int64_t)be) return 0;
    return (size_t)(n / (int64_t)be) * bb;
}

const char *ggml_type_name(uint32_t t) {
    switch (t) {
        case GGML_F32: return "f32";
        case GGML_F16: return "f16";
        case GGML_BF16: return "bf16";
        case GGML_I8: return "i8";
        case GGML_I16: return "i16";
        case GGML_I32: return "i32";
        case GGML_Q4_0: return "q4_0";
        case GGML_Q5_0: return "q5_0";
        case GGML_Q8_0: return "q8_0";
        case GGML_Q4_K: return "q4_K";
        case GGML_Q6_K: return "q6_K";
        case GGML_Q8_K: return "q8_K";
        default: return "?";
    }
}

namespace {

struct Cursor {
    const uint8_t *p, *end;
    bool ok = true;
    template <class T>
    T rd() {
        T v{};
        if ((size_t)(end - p) < sizeof(T)) {
            ok = false;
            return v;
        }
        std::memcpy(&v, p, sizeof(T));
        p += sizeof(T);
        return v;
    }
    std::string str() {
        uint64_t n = rd<uint64_t>();
        if (!ok || (uint64_t)(end - p) < n) {
            ok = false;
            return {};
        }
        std::string s((const char *)p, n);
        p += n;
        return s;
    }
};

bool read_scalar(Cursor &c, uint32_t type, GgufValue &v) {
    switch (type) {
        case GGUF_U8: v.u = c.rd<uint8_t>(); break;
        case GGUF_I8: v.u = (uint64_t)(int64_t)c.rd<int8_t>(); break;
        case GGUF_U16: v.u = c.rd<uint16_t>(); break;
        case GGUF_I16: v.u = (uint64_t)(int64_t)c.rd<int16_t>(); break;
        case GGUF_U32: v.u = c.rd<uint32_t>(); break;
        case GGUF_I32: v.u = (uint64_t)(int64_t)c.rd<int32_t>(); break;
        case GGUF_U64: v.u = c.rd<uint64_t>(); break;
        case GGUF_I64: v.u = (uint64_t)c.rd<int64_t>(); break;
        case GGUF_BOOL: v.u = c.rd<uint8_t>() ? 1 : 0; break;
        case GGUF_F32: v.f = c.rd<float>(); break;
        case GGUF_F64: v.f = c.rd<double>(); break;
        case GGUF_STR: v.s = c.str(); break;
        default: return false;
    }
    if (type != GGUF_F32 && type != GGUF_F64 && type != GGUF_STR) v.f = (double)(int64_t)v.u;
    // the integer view of a float value: only where it is representable (NaN / inf / huge -> 0)
    if (type == GGUF_F32 || type == GGUF_F64)
        v.u = std::isfinite(v.f) && std::fabs(v.f) < 9.0e18 ? (uint64_t)(int64_t)v.f : 0;
    return c.ok;
}

}  // namespace

GgufFile::~GgufFile() { close(); }

void GgufFile::close() {
    if (map_) munmap(map_, map_size_);
    map_ = nullptr;
    map_size_ = 0;
    kv_.clear();
    tensors_.clear();
    index_.clear();
}

bool GgufFile::open(const std::string &path) {
    close();
    path_ = path;
    int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) {
        set_error("gguf: cannot open %s", path.c_str());
        return false;
    }
    struct stat st;
    if (fstat(fd, &st) != 0 || st.st_size < 24) {
        ::close(fd);
        set_error("gguf: %s too small", path.c_str());
        return false;
    }
    map_size_ = (size_t)st.st_size;
    map_ = mmap(nullptr, map_size_, PROT_READ, MAP_PRIVATE, fd, 0);
    ::close(fd);
    if (map_ == MAP_FAILED) {
        map_ = nullptr;
        set_error("gguf: mmap %s failed", path.c_str());
        return false;
    }
    const uint8_t *base = (const uint8_t *)map_;
    Cursor c{base, base + map_size_};
    const uint32_t magic = c.rd<uint32_t>();
    const uint32_t version = c.rd<uint32_t>();
    if (magic != 0x46554747u || (version != 2 && version != 3)) {
        set_error("gguf: %s is not GGUF v2/v3 (magic %08x version %u)", path.c_str(), magic,
                  version);
        close();
        return false;
    }
    const uint64_t n_tensors = c.rd<uint64_t>();
    const uint64_t n_kv = c.rd<uint64_t>();
    for (uint64_t i = 0; i < n_kv && c.ok; ++i) {
        std::string key = c.str();
        GgufValue v;
        v.type = c.rd<uint32_t>();
        if (v.type == GGUF_ARR) {
            v.arr_type = c.rd<uint32_t>();
            const uint64_t n = c.rd<uint64_t>();
            if (!c.ok || n > map_size_) {
                c.ok = false;
                break;
            }
            for (uint64_t j = 0; j < n && c.ok; ++j) {
                GgufValue e;
                if (!read_scalar(c, v.arr_type, e)) {
                    c.ok = false;
                    break;
                }
                if (v.arr_type == GGUF_STR)
                    v.arr_s.push_back(std::move(e.s));
                else if (v.arr_type == GGUF_F32 || v.arr_type == GGUF_F64)
                    v.arr_f.push_back(e.f);
                else
                    v.arr_i.push_back((int64_t)e.u);
            }
        } else if (!read_scalar(c, v.type, v)) {
            c.ok = false;
        }
        kv_[key] = std::move(v);
    }
    for (uint64_t i = 0; i < n_tensors && c.ok; ++i) {
        GgufTensor t;
        t.name = c.str();
        t.n_dims = (int)c.rd<uint32_t>();
        if (t.n_dims < 1 || t.n_dims > 4) {
            c.ok = false;
            break;
        }
        // every dimension in [0, 2^40) and the byte count without overflow (a hostile file
        // must not wrap the bounds check below)
        bool shape_ok = true;
        for (int d = 0; d < t.n_dims; ++d) {
            const uint64_t v = c.rd<uint64_t>();
            shape_ok = shape_ok && v < (1ull << 40);
            t.ne[d] = shape_ok ? (int64_t)v : 0;
        }
        t.type = c.rd<uint32_t>();
        t.offset = c.rd<uint64_t>();
        uint64_t rows = 0, nb = 0;
        if (shape_ok && !__builtin_mul_overflow((uint64_t)t.ne[1], (uint64_t)t.ne[2], &rows) &&
            !__builtin_mul_overflow(rows, (uint64_t)t.ne[3], &rows) &&
            !__builtin_mul_overflow((uint64_t)ggml_row_bytes(t.type, t.ne[0]), rows, &nb))
            t.nbytes = (size_t)nb;
        if (!c.ok) break;
        if (!t.nbytes) {
            set_error("gguf: tensor %s has unsupported type %u / shape", t.name.c_str(), t.type);
            close();
            return false;
        }
        index_[t.name] = tensors_.size();
        tensors_.push_back(std::move(t));
    }
    if (!c.ok) {
        set_error("gguf: truncated header in %s", path.c_str());
        close();
        return false;
    }
    const int64_t align = get_int("general.alignment", 32);
    if (align < 1 || align > (1 << 20) || (align & (align - 1))) {
        set_error("gguf: %s has general.alignment %lld (a power of two is required)", path.c_str(), (long long)align);
        close();
        return false;
    }
    size_t off = (size_t)(c.p - base);
    data_offset_ = (off + (size_t)align - 1) / (size_t)align * (size_t)align;
    for (auto &t : tensors_) {
        // overflow-safe: data_offset_ + offset + nbytes <= map_size_
        if (data_offset_ > map_size_ || t.offset > map_size_ - data_offset_ ||
            t.nbytes > map_size_ - data_offset_ - t.offset) {
            set_error("gguf: tensor %s data out of file bounds", t.name.c_str());
            close();
            return false;
        }
        t.data = base + data_offset_ + t.offset;
    }
    return true;
}

const GgufValue *GgufFile::get(const std::string &key) const {
    auto it = kv_.find(key);
    return it == kv_.end() ? nullptr : &it->second;
}

int64_t GgufFile::get_int(const std::string &key, int64_t def) const {
    const GgufValue *v = get(key);
    if (!v || v->type == GGUF_STR || v->type == GGUF_ARR) return def;
    return (int64_t)v->u;
}

double GgufFile::get_float(const std::string &key, double def) const {
    const GgufValue *v = get(key);
    if (!v || v->type == GGUF_STR || v->type == GGUF_ARR) return def;
    return v->f;
}

std::string GgufFile::get_str(const std::string &key, const std::string &def) const {
    const GgufValue *v = get(key);
    return (v && v->type == GGUF_STR) ? v->s : def;
}

const GgufTensor *GgufFile::tensor(const std::string &name) const {
    auto it = index_.find(name);
    return it == index_.end() ? nullptr : &tensors_[it->second];
}

// ---------------- writer ----------------
namespace {
template <class T>
void put(std::vector<uint8_t> &b, T v) {
    const uint8_t *p = (const uint8_t *)&v;
    b.insert(b.end(), p, p + sizeof(T));
}
void put_str(std::vector<uint8_t> &b, const std::string &s) {
    put<uint64_t>(b, s.size());
    b.insert(b.end(), s.begin(), s.end());
}
}  // namespace

void GgufWriter::kv_u32(const std::string &k, uint32_t v) {
    put_str(kvbuf_, k), put<uint32_t>(kvbuf_, GGUF_U32), put<uint32_t>(kvbuf_, v), ++n_kv_;
}
void GgufWriter::kv_i32(const std::string &k, int32_t v) {
    put_str(kvbuf_, k), put<uint32_t>(kvbuf_, GGUF_I32), put<int32_t>(kvbuf_, v), ++n_kv_;
}
void GgufWriter::kv_f32(const std::string &k, float v) {
    put_str(kvbuf_, k), put<uint32_t>(kvbuf_, GGUF_F32), put<float>(kvbuf_, v), ++n_kv_;
}
void GgufWriter::kv_bool(const std::string &k, bool v) {
    put_str(kvbuf_, k), put<uint32_t>(kvbuf_, GGUF_BOOL), put<uint8_t>(kvbuf_, v ? 1 : 0), ++n_kv_;
}
void GgufWriter::kv_str(const std::string &k, const std::string &v) {
    put_str(kvbuf_, k), put<uint32_t>(kvbuf_, GGUF_STR), put_str(kvbuf_, v), ++n_kv_;
}
void GgufWriter::kv_arr_str(const std::string &k, const std::vector<std::string> &v) {
    put_str(kvbuf_, k), put<uint32_t>(kvbuf_, GGUF_ARR), put<uint32_t>(kvbuf_, GGUF_STR);
    put<uint64_t>(kvbuf_, v.size());
    for (auto &s : v) put_str(kvbuf_, s);
    ++n_kv_;
}
void GgufWriter::kv_arr_i32(const std::string &k, const std::vector<int32_t> &v) {
    put_str(kvbuf_, k), put<uint32_t>(kvbuf_, GGUF_ARR), put<uint32_t>(kvbuf_, GGUF_I32);
    put<uint64_t>(kvbuf_, v.size());
    for (auto x : v) put<int32_t>(kvbuf_, x);
    ++n_kv_;
}
void GgufWriter::kv_arr_f32(const std::string &k, const std::vector<float> &v) {
    put_str(kvbuf_, k), put<uint32_t>(kvbuf_, GGUF_ARR), put<uint32_t>(kvbuf_, GGUF_F32);
    put<uint64_t>(kvbuf_, v.size());
    for (auto x : v) put<float>(kvbuf_, x);
    ++n_kv_;
}

void GgufWriter::add_tensor(const std::string &name, uint32_t type, std::vector<int64_t> ne) {
    T t;
    t.name = name;
    t.type = type;
    t.ne = ne;
    int64_t rows = 1;
    for (size_t i = 1; i < ne.size(); ++i) rows *= ne[i];
    t.nbytes = ggml_row_bytes(type, ne[0]) * (size_t)rows;
    const uint64_t align = 32;
    t.offset = (data_size_ + align - 1) / align * align;
    data_size_ = t.offset + t.nbytes;
    tensors_.push_back(std::move(t));
}

bool GgufWriter::write_header(FILE *f) const {
    std::vector<uint8_t> h;
    put<uint32_t>(h, 0x46554747u);
    put<uint32_t>(h, 3);
    put<uint64_t>(h, tensors_.size());
    put<uint64_t>(h, n_kv_);
    h.insert(h.end(), kvbuf_.begin(), kvbuf_.end());
    for (auto &t : tensors_) {
        put_str(h, t.name);
        put<uint32_t>(h, (uint32_t)t.ne.size());
        for (auto n : t.ne) put<uint64_t>(h, (uint64_t)n);
        put<uint32_t>(h, t.type);
        put<uint64_t>(h, t.offset);
    }
    while (h.size() % 32) h.push_back(0);
    return std::fwrite(h.data(), 1, h.size(), f) == h.size();
}

}  // namespace mio
