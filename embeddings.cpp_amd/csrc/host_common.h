// Host-side shared definitions for libbert.so (no HIP types here).
#pragma once

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace emb {

// Weight storage formats = the ggml type ids the reference file format stores
// per tensor (bert.cpp:720-742).  8 (q8_0) is this build's extension.
enum WFmt : int32_t { FMT_F32 = 0, FMT_F16 = 1, FMT_Q4_0 = 2, FMT_Q4_1 = 3, FMT_Q8_0 = 8 };

constexpr int QK = 32;  // elements per quant block

inline bool fmt_valid(int f) { return f == FMT_F32 || f == FMT_F16 || f == FMT_Q4_0 || f == FMT_Q4_1 || f == FMT_Q8_0; }

// bytes per block of 32 elements (f32/f16 counted per 32 elements too)
inline size_t fmt_block_bytes(int f)
{
    switch (f) {
    case FMT_F32: return 128;
    case FMT_F16: return 64;
    case FMT_Q4_0: return 18;   // fp16 d + 16 nibble bytes
    case FMT_Q4_1: return 20;   // fp16 d + fp16 m + 16 nibble bytes
    case FMT_Q8_0: return 34;   // fp16 d + 32 int8
    default: return 0;
    }
}

inline size_t fmt_row_bytes(int f, int64_t k) { return fmt_block_bytes(f) * (size_t)(k / QK); }

// IEEE binary16 conversions, round-to-nearest-even (the rounding numpy's
// astype(float16) in convert-to-ggml.py and F16C use).
uint16_t f32_to_f16(float f);
float f16_to_f32(uint16_t h);
// The era's 65536-entry fp16 GELU and exp tables (model_file.cpp).
void era_tables(std::vector<uint16_t> &gelu, std::vector<uint16_t> &ex);

struct HParams {
    int32_t n_vocab = 0, n_max_tokens = 0, n_embd = 0, n_intermediate = 0, n_head = 0, n_layer = 0, ftype = 0;
};

struct HostTensor {
    int32_t fmt = -1;
    int32_t ne0 = 0, ne1 = 1;       // ne0 = fastest (in-features)
    std::vector<uint8_t> bytes;     // exactly as stored in the file
    bool present() const { return fmt >= 0; }
};

struct HostLayer {
    HostTensor q_w, k_w, v_w, o_w, i_w, o2_w;
    HostTensor q_b, k_b, v_b, o_b, i_b, o2_b;
    HostTensor ln_att_w, ln_att_b, ln_out_w, ln_out_b;
};

struct HostModel {
    HParams hp;
    std::vector<std::string> vocab;
    HostTensor word, ttype, pos, ln_e_w, ln_e_b;
    std::vector<HostLayer> layers;
    size_t total_bytes = 0;
    int n_tensors = 0;
};

// Parse a model file in the reference format (bert.cpp:423-766).  On failure
// returns false with a message in err (the caller prints it to stderr).
bool load_model_file(const char *path, HostModel &m, std::string &err, bool verbose);

// Message sink (log.cpp): errorf prints to stderr and appends the line to
// BERT_LOG=<file> when set (one unbuffered write per line); trace writes to the
// BERT_LOG file only (the load path's stages); infof prints to stdout only.  fault_inject(stage): true when the test-only
// BERT_FAULT_INJECT list names `stage`.
void errorf(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
void infof(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
void trace(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
bool fault_inject(const char *stage);

// Dequantize one row of k elements into f32.
void dequant_row(int fmt, const uint8_t *src, float *dst, int64_t k);
// One row of k values in file format `fmt` (the quantizer's block rules).
void quantize_row(int fmt, const float *x, uint8_t *dst, int64_t k);

// Native quantizer (mirrors models/quantize.cpp:27-268; itype 2, 3, or 8).
int quantize_file(const char *in, const char *out, int itype, bool verbose);
// HF directory (config.json, vocab.txt, model.safetensors) -> model file (converter.cpp)
int convert_hf_dir(const std::string &dir, const std::string &fname_out, int ftype);

}  // namespace emb
