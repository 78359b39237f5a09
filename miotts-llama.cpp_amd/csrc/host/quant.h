// ggml block quant formats (public ggml spec) on the host:
// fp16 conversion, row quantizers (used to make synthetic Q8_0 / Q4_K_M models),
// row dequantizers (embedding get_rows), and the re-layout of a GGUF quantized matrix
// into the "split" layout the gfx950 matvec kernels stream:
//
//   Q8_0 : qs [R][K]      int8          | d  [R][K/32]  f16
//   Q4_K : qs [R][K/2]    u8 nibbles    | hd [R][K/256] 16 B = {d, dmin, 4 x 24-bit scale pairs}
//   Q6_K : ql [R][K/2]    u8            | qh [R][K/4] u8 | sc [R][K/16] i8 (lane-pair order) | d [R][K/256] f16
//
// Same bytes per weight as GGUF (algorithmic bytes unchanged); each row's quant payload
// becomes one contiguous, 16-B aligned run, so one wave reads a row with 16 B per lane.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace mio {

#pragma pack(push, 1)
struct BlockQ8_0 {
    uint16_t d;
    int8_t qs[32];
};
// llama-quantize's fallbacks for rows whose length is not a multiple of 256 (Q4_K -> Q5_0,
// llama.cpp llama-quant.cpp) and plain Q4_0 files: 32 weights per block, codes q - 8 / q - 16.
struct BlockQ4_0 {
    uint16_t d;
    uint8_t qs[16];
};
struct BlockQ5_0 {
    uint16_t d;
    uint8_t qh[4];
    uint8_t qs[16];
};
struct BlockQ4_K {
    uint16_t d, dmin;
    uint8_t scales[12];
    uint8_t qs[128];
};
struct BlockQ6_K {
    uint8_t ql[128];
    uint8_t qh[64];
    int8_t scales[16];
    uint16_t d;
};
#pragma pack(pop)
static_assert(sizeof(BlockQ8_0) == 34, "q8_0");
static_assert(sizeof(BlockQ4_0) == 18, "q4_0");
static_assert(sizeof(BlockQ5_0) == 22, "q5_0");
static_assert(sizeof(BlockQ4_K) == 144, "q4_K");
static_assert(sizeof(BlockQ6_K) == 210, "q6_K");

float fp16_to_f32(uint16_t h);
uint16_t f32_to_fp16(float f);  // round to nearest even
uint16_t f32_to_bf16(float f);  // ggml_compute_fp32_to_bf16

void quantize_row_q8_0(const float *x, void *y, int64_t k);
void quantize_row_q4_0(const float *x, void *y, int64_t k);
void quantize_row_q5_0(const float *x, void *y, int64_t k);
void quantize_row_q4_K(const float *x, void *y, int64_t k);
void quantize_row_q6_K(const float *x, void *y, int64_t k);
bool quantize_row(uint32_t type, const float *x, void *y, int64_t k);
bool dequantize_row(uint32_t type, const void *x, float *y, int64_t k);

// Q4_0 / Q5_0 rows as Q8_0 rows, losslessly: a block's codes x - 8 (Q4_0) or x - 16 (Q5_0)
// lie in [-16, 15] and keep their f16 scale, and ggml's vec_dot_q4_0_q8_0 / vec_dot_q5_0_q8_0
// (vec_dot_type Q8_0, sumi * (d_w * d_a) per block) equal vec_dot_q8_0_q8_0 on the repacked
// block term for term, as dequantize_row does. dst: R * (K / 32) * 34 bytes.
bool repack_to_q8_0(uint32_t type, const void *src, int64_t rows, int64_t k, void *dst);
bool repacks_to_q8_0(uint32_t type);

// Split layout of one [R][K] matrix (offsets in bytes from the tensor's base).
struct SplitLayout {
    uint32_t type = 0;
    int64_t rows = 0, k = 0;
    size_t off[4] = {0, 0, 0, 0};
    size_t bytes = 0;
};
SplitLayout split_layout(uint32_t type, int64_t rows, int64_t k);
// GGUF rows -> split layout (dst has layout.bytes). Returns false on unsupported type.
bool to_split(uint32_t type, const void *src, int64_t rows, int64_t k, uint8_t *dst);

}  // namespace mio
