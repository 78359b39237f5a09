// GGUF v2/v3 reader (mmap) and writer — our own implementation of the public GGUF
// container format that the reference reads through gguf_init_from_file
// (miocodec.cpp:430-431, :818-834) and llama_model_load_from_file
// (test-to-speech.cpp:47-49). Tensor data offsets = data_offset + tensor offset
// (miocodec.cpp:99,122).
#pragma once

#include <cstddef>
#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace mio {

// ggml tensor type ids (public ggml enum values).
enum GgmlType : uint32_t {
    GGML_F32 = 0,
    GGML_F16 = 1,
    GGML_Q4_0 = 2,
    GGML_Q5_0 = 6,
    GGML_Q8_0 = 8,
    GGML_Q4_K = 12,
    GGML_Q6_K = 14,
    GGML_Q8_K = 15,
    GGML_I8 = 24,
    GGML_I16 = 25,
    GGML_I32 = 26,
    GGML_BF16 = 30,
};

// bytes per block / elements per block for the supported types
size_t ggml_type_block_bytes(uint32_t t);
size_t ggml_type_block_elems(uint32_t t);
size_t ggml_row_bytes(uint32_t t, int64_t n_elems);
const char *ggml_type_name(uint32_t t);

enum GgufValType : uint32_t {
    GGUF_U8 = 0, GGUF_I8 = 1, GGUF_U16 = 2, GGUF_I16 = 3, GGUF_U32 = 4, GGUF_I32 = 5,
    GGUF_F32 = 6, GGUF_BOOL = 7, GGUF_STR = 8, GGUF_ARR = 9, GGUF_U64 = 10, GGUF_I64 = 11,
    GGUF_F64 = 12,
};

struct GgufValue {
    uint32_t type = 0;
    uint32_t arr_type = 0;
    uint64_t u = 0;  // integer / bool payload (sign-extended for signed types)
    double f = 0;    // float payload
    std::string s;
    std::vector<std::string> arr_s;
    std::vector<int64_t> arr_i;
    std::vector<double> arr_f;
};

struct GgufTensor {
    std::string name;
    uint32_t type = 0;
    int n_dims = 0;
    int64_t ne[4] = {1, 1, 1, 1};
    uint64_t offset = 0;  // relative to data section
    size_t nbytes = 0;
    const uint8_t *data = nullptr;  // into the mapping
    int64_t nelements() const { return ne[0] * ne[1] * ne[2] * ne[3]; }
};

class GgufFile {
public:
    GgufFile() = default;
    ~GgufFile();
    GgufFile(const GgufFile &) = delete;
    GgufFile &operator=(const GgufFile &) = delete;

    bool open(const std::string &path);  // false + mio::set_error on failure
    void close();

    bool has(const std::string &key) const { return kv_.count(key) != 0; }
    const GgufValue *get(const std::string &key) const;
    int64_t get_int(const std::string &key, int64_t def) const;
    double get_float(const std::string &key, double def) const;
    std::string get_str(const std::string &key, const std::string &def = "") const;

    const GgufTensor *tensor(const std::string &name) const;
    const std::vector<GgufTensor> &tensors() const { return tensors_; }
    size_t data_offset() const { return data_offset_; }
    const std::string &path() const { return path_; }

private:
    std::string path_;
    std::map<std::string, GgufValue> kv_;
    std::vector<GgufTensor> tensors_;
    std::map<std::string, size_t> index_;
    size_t data_offset_ = 0;
    void *map_ = nullptr;
    size_t map_size_ = 0;
};

// Streaming GGUF v3 writer: add KVs and tensor descriptors first, then write().
class GgufWriter {
public:
    void kv_u32(const std::string &k, uint32_t v);
    void kv_i32(const std::string &k, int32_t v);
    void kv_f32(const std::string &k, float v);
    void kv_bool(const std::string &k, bool v);
    void kv_str(const std::string &k, const std::string &v);
    void kv_arr_str(const std::string &k, const std::vector<std::string> &v);
    void kv_arr_i32(const std::string &k, const std::vector<int32_t> &v);
    void kv_arr_f32(const std::string &k, const std::vector<float> &v);
    // Tensor whose bytes are produced later by `fill(dst, nbytes)`; ne in ggml order.
    void add_tensor(const std::string &name, uint32_t type, std::vector<int64_t> ne);
    // Writes header + tensor infos; then calls fill(i, dst, nbytes) per tensor in order.
    template <class Fill>
    bool write(const std::string &path, Fill fill);

    struct T {
        std::string name;
        uint32_t type;
        std::vector<int64_t> ne;
        size_t nbytes;
        uint64_t offset;
    };
    const std::vector<T> &tensors() const { return tensors_; }

private:
    std::vector<uint8_t> kvbuf_;
    uint64_t n_kv_ = 0;
    std::vector<T> tensors_;
    uint64_t data_size_ = 0;
    bool write_header(FILE *f) const;
};

}  // namespace mio

#include <cstdio>

template <class Fill>
bool mio::GgufWriter::write(const std::string &path, Fill fill) {
    FILE *f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    if (!write_header(f)) {
        std::fclose(f);
        return false;
    }
    std::vector<uint8_t> buf;
    uint64_t pos = 0;
    for (size_t i = 0; i < tensors_.size(); ++i) {
        const T &t = tensors_[i];
        if (t.offset > pos) {
            std::vector<uint8_t> pad(t.offset - pos, 0);
            std::fwrite(pad.data(), 1, pad.size(), f);
            pos = t.offset;
        }
        buf.assign(t.nbytes, 0);
        fill(i, buf.data(), t.nbytes);
        if (std::fwrite(buf.data(), 1, t.nbytes, f) != t.nbytes) {
            std::fclose(f);
            return false;
        }
        pos += t.nbytes;
    }
    return std::fclose(f) == 0;
}
