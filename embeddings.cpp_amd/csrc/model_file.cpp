// Reference-format model reader + native quantizer (host C++).
//
// File layout (reference bert.cpp:434-766, writer models/convert-to-ggml.py:68-108):
//   u32 magic 0x67676d6c
//   i32 n_vocab, n_max_tokens, n_embd, n_intermediate, n_head, n_layer, ftype
//   n_vocab x { u32 len; u8 bytes[len] }
//   until EOF: { i32 n_dims; i32 name_len; i32 ftype; i32 ne[n_dims]; name; data }
// 1-D tensors are f32; 2-D "*weight" tensors are in the header ftype.
#include "host_common.h"

#include <cmath>
#include <cstdio>
#include <memory>

namespace emb {

uint16_t f32_to_f16(float f)
{
    uint32_t x;
    std::memcpy(&x, &f, 4);
    const uint32_t sign = (x >> 16) & 0x8000u;
    const int32_t e = (int32_t)((x >> 23) & 0xffu);
    uint32_t m = x & 0x7fffffu;
    if (e == 255) return (uint16_t)(sign | 0x7c00u | (m ? 0x200u : 0u));
    const int32_t he = e - 112;  // rebias 127 -> 15
    if (he >= 31) return (uint16_t)(sign | 0x7c00u);
    if (he <= 0) {
        if (he < -10) return (uint16_t)sign;
        m |= 0x800000u;
        const int sh = 14 - he;
        uint32_t q = m >> sh;
        const uint32_t r = m & ((1u << sh) - 1u), half = 1u << (sh - 1);
        q += (r > half || (r == half && (q & 1u))) ? 1u : 0u;
        return (uint16_t)(sign | q);
    }
    uint32_t h = sign | ((uint32_t)he << 10) | (m >> 13);
    const uint32_t r = m & 0x1fffu;
    h += (r > 0x1000u || (r == 0x1000u && (h & 1u))) ? 1u : 0u;
    return (uint16_t)h;
}

float f16_to_f32(uint16_t h)
{
    const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    const uint32_t e = (h >> 10) & 0x1fu, m = h & 0x3ffu;
    uint32_t u;
    if (e == 0) {
        if (m == 0) { u = sign; }
        else { float v = (float)m * 5.9604644775390625e-08f; return sign ? -v : v; }
    } else if (e == 31) {
        u = sign | 0x7f800000u | (m << 13);
    } else {
        u = sign | ((e + 112) << 23) | (m << 13);
    }
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

// The ggml-era fp16 function tables bert.cpp's GELU and softmax exp read
// (GGML_GELU_FP16 / the fp16 exp table, bert.cpp:1025, 1063): entry i = f16 of the
// f32 function at the f16 value i, built once on the host with libm, as ggml did
// at ggml_init.  The f32 chain (f32.hip) indexes them by the f16 bit pattern.
void era_tables(std::vector<uint16_t> &gelu, std::vector<uint16_t> &ex)
{
    gelu.resize(65536);
    ex.resize(65536);
    const float k_a = 0.044715f, k_s = 0.79788456080286535587989211986876f;   // sqrt(2/pi)
    for (uint32_t i = 0; i < 65536u; ++i) {
        const float f = f16_to_f32((uint16_t)i);
        const float g = 0.5f * f * (1.0f + std::tanh(k_s * f * (1.0f + k_a * f * f)));
        gelu[i] = f32_to_f16(g);
        ex[i] = f32_to_f16(std::exp(f));
    }
}

void dequant_row(int fmt, const uint8_t *src, float *dst, int64_t k)
{
    const int64_t nb = k / QK;
    switch (fmt) {
    case FMT_F32: std::memcpy(dst, src, (size_t)k * 4); break;
    case FMT_F16:
        for (int64_t i = 0; i < k; ++i) { uint16_t h; std::memcpy(&h, src + 2 * i, 2); dst[i] = f16_to_f32(h); }
        break;
    case FMT_Q4_0:
        for (int64_t b = 0; b < nb; ++b) {
            const uint8_t *p = src + b * 18;
            uint16_t dh; std::memcpy(&dh, p, 2);
            const float d = f16_to_f32(dh);
            for (int j = 0; j < 16; ++j) {
                dst[b * 32 + j] = (float)((p[2 + j] & 15) - 8) * d;
                dst[b * 32 + 16 + j] = (float)((p[2 + j] >> 4) - 8) * d;
            }
        }
        break;
    case FMT_Q4_1:
        for (int64_t b = 0; b < nb; ++b) {
            const uint8_t *p = src + b * 20;
            uint16_t dh, mh; std::memcpy(&dh, p, 2); std::memcpy(&mh, p + 2, 2);
            const float d = f16_to_f32(dh), mn = f16_to_f32(mh);
            for (int j = 0; j < 16; ++j) {
                dst[b * 32 + j] = (float)(p[4 + j] & 15) * d + mn;
                dst[b * 32 + 16 + j] = (float)(p[4 + j] >> 4) * d + mn;
            }
        }
        break;
    case FMT_Q8_0:
        for (int64_t b = 0; b < nb; ++b) {
            const uint8_t *p = src + b * 34;
            uint16_t dh; std::memcpy(&dh, p, 2);
            const float d = f16_to_f32(dh);
            for (int j = 0; j < 32; ++j) dst[b * 32 + j] = (float)(int8_t)p[2 + j] * d;
        }
        break;
    default: break;
    }
}

namespace {

struct File {
    FILE *f = nullptr;
    explicit File(const char *p, const char *mode) : f(std::fopen(p, mode)) {}
    ~File() { if (f) std::fclose(f); }
    bool read(void *p, size_t n) { return std::fread(p, 1, n, f) == n; }
    bool write(const void *p, size_t n) { return std::fwrite(p, 1, n, f) == n; }
};

// Expected shape and destination of every tensor name (bert.cpp:595-645).
HostTensor *slot(HostModel &m, const std::string &name, int32_t &e0, int32_t &e1, bool &vec)
{
    const int32_t d = m.hp.n_embd, f = m.hp.n_intermediate;
    vec = false;
    if (name == "embeddings.word_embeddings.weight") { e0 = d; e1 = m.hp.n_vocab; return &m.word; }
    if (name == "embeddings.token_type_embeddings.weight") { e0 = d; e1 = 2; return &m.ttype; }
    if (name == "embeddings.position_embeddings.weight") { e0 = d; e1 = m.hp.n_max_tokens; return &m.pos; }
    vec = true; e1 = 1;
    if (name == "embeddings.LayerNorm.weight") { e0 = d; return &m.ln_e_w; }
    if (name == "embeddings.LayerNorm.bias") { e0 = d; return &m.ln_e_b; }
    static const std::string pre = "encoder.layer.";
    if (name.compare(0, pre.size(), pre) != 0) return nullptr;
    size_t pos = pre.size(), end = name.find('.', pos);
    if (end == std::string::npos) return nullptr;
    int l = -1;
    try { l = std::stoi(name.substr(pos, end - pos)); } catch (...) { return nullptr; }
    if (l < 0 || l >= m.hp.n_layer || std::to_string(l) != name.substr(pos, end - pos)) return nullptr;
    HostLayer &L = m.layers[(size_t)l];
    const std::string s = name.substr(end + 1);
    struct Row { const char *n; bool vec; int32_t e0, e1; HostTensor *t; };
    const Row rows[] = {
        {"attention.self.query.weight", false, d, d, &L.q_w}, {"attention.self.query.bias", true, d, 1, &L.q_b},
        {"attention.self.key.weight", false, d, d, &L.k_w},   {"attention.self.key.bias", true, d, 1, &L.k_b},
        {"attention.self.value.weight", false, d, d, &L.v_w}, {"attention.self.value.bias", true, d, 1, &L.v_b},
        {"attention.output.dense.weight", false, d, d, &L.o_w}, {"attention.output.dense.bias", true, d, 1, &L.o_b},
        {"attention.output.LayerNorm.weight", true, d, 1, &L.ln_att_w},
        {"attention.output.LayerNorm.bias", true, d, 1, &L.ln_att_b},
        {"intermediate.dense.weight", false, d, f, &L.i_w}, {"intermediate.dense.bias", true, f, 1, &L.i_b},
        {"output.dense.weight", false, f, d, &L.o2_w},       {"output.dense.bias", true, d, 1, &L.o2_b},
        {"output.LayerNorm.weight", true, d, 1, &L.ln_out_w}, {"output.LayerNorm.bias", true, d, 1, &L.ln_out_b},
    };
    for (const Row &r : rows)
        if (s == r.n) { vec = r.vec; e0 = r.e0; e1 = r.e1; return r.t; }
    return nullptr;
}

}  // namespace

bool load_model_file(const char *path, HostModel &m, std::string &err, bool verbose)
{
    File fp(path, "rb");
    if (!fp.f) { err = std::string("failed to open '") + path + "'"; return false; }
    uint32_t magic = 0;
    if (!fp.read(&magic, 4) || magic != 0x67676d6cu) {
        err = std::string("invalid model file '") + path + "' (bad magic)";
        return false;
    }
    int32_t hp[7];
    if (!fp.read(hp, sizeof(hp))) { err = "truncated header"; return false; }
    m.hp.n_vocab = hp[0]; m.hp.n_max_tokens = hp[1]; m.hp.n_embd = hp[2]; m.hp.n_intermediate = hp[3];
    m.hp.n_head = hp[4]; m.hp.n_layer = hp[5]; m.hp.ftype = hp[6];
    if (verbose) {
        std::printf("bert_load_from_file: n_vocab = %d\n", m.hp.n_vocab);
        std::printf("bert_load_from_file: n_max_tokens   = %d\n", m.hp.n_max_tokens);
        std::printf("bert_load_from_file: n_embd  = %d\n", m.hp.n_embd);
        std::printf("bert_load_from_file: n_intermediate  = %d\n", m.hp.n_intermediate);
        std::printf("bert_load_from_file: n_head  = %d\n", m.hp.n_head);
        std::printf("bert_load_from_file: n_layer = %d\n", m.hp.n_layer);
        std::printf("bert_load_from_file: f16     = %d\n", m.hp.ftype);
    }
    if (m.hp.n_vocab <= 0 || m.hp.n_embd <= 0 || m.hp.n_layer <= 0 || m.hp.n_head <= 0 ||
        m.hp.n_max_tokens <= 0 || m.hp.n_intermediate <= 0 || m.hp.n_embd % m.hp.n_head != 0) {
        err = "invalid hparams";
        return false;
    }
    if (!fmt_valid(m.hp.ftype)) {
        err = std::string("invalid model file '") + path + "' (bad f16 value " + std::to_string(m.hp.ftype) + ")";
        return false;
    }
    m.vocab.resize((size_t)m.hp.n_vocab);
    for (int32_t i = 0; i < m.hp.n_vocab; ++i) {
        uint32_t len = 0;
        if (!fp.read(&len, 4) || len > (1u << 20)) { err = "truncated vocab"; return false; }
        m.vocab[(size_t)i].resize(len);
        if (len && !fp.read(&m.vocab[(size_t)i][0], len)) { err = "truncated vocab"; return false; }
    }
    m.layers.assign((size_t)m.hp.n_layer, HostLayer());
    for (;;) {
        int32_t h3[3];
        if (!fp.read(h3, sizeof(h3))) break;
        const int32_t n_dims = h3[0], name_len = h3[1], fmt = h3[2];
        int32_t ne[2] = {1, 1};
        if (n_dims < 1 || n_dims > 2 || !fp.read(ne, 4 * (size_t)n_dims) || name_len <= 0 || name_len > 4096) {
            err = "bad tensor record";
            return false;
        }
        std::string name((size_t)name_len, '\0');
        if (!fp.read(&name[0], (size_t)name_len)) { err = "truncated tensor name"; return false; }
        int32_t e0 = 0, e1 = 0;
        bool vec = false;
        HostTensor *t = slot(m, name, e0, e1, vec);
        if (!t) { err = "unknown tensor '" + name + "' in model file"; return false; }
        if (ne[0] != e0 || ne[1] != e1) { err = "tensor '" + name + "' has wrong shape in model file"; return false; }
        if (!fmt_valid(fmt)) { err = "unknown ftype " + std::to_string(fmt) + " in model file"; return false; }
        if (vec && fmt != FMT_F32) { err = "tensor '" + name + "' must be f32"; return false; }
        if (!vec && fmt != m.hp.ftype) {
            err = "tensor '" + name + "' has wrong size in model file";
            return false;
        }
        if (fmt != FMT_F32 && fmt != FMT_F16 && ne[0] % QK != 0) { err = "tensor '" + name + "' not block aligned"; return false; }
        t->fmt = fmt; t->ne0 = ne[0]; t->ne1 = ne[1];
        t->bytes.resize(fmt_row_bytes(fmt, ne[0]) * (size_t)ne[1]);
        if (!fp.read(t->bytes.data(), t->bytes.size())) { err = "truncated data for '" + name + "'"; return false; }
        m.total_bytes += t->bytes.size();
        ++m.n_tensors;
    }
    auto need = [&](const HostTensor &t, const char *what) {
        if (!t.present()) { err = std::string("missing tensor ") + what; return false; }
        return true;
    };
    if (!need(m.word, "word_embeddings") || !need(m.ttype, "token_type_embeddings") || !need(m.pos, "position_embeddings") ||
        !need(m.ln_e_w, "embeddings.LayerNorm.weight") || !need(m.ln_e_b, "embeddings.LayerNorm.bias"))
        return false;
    for (int l = 0; l < m.hp.n_layer; ++l) {
        HostLayer &L = m.layers[(size_t)l];
        const HostTensor *all[] = {&L.q_w, &L.k_w, &L.v_w, &L.o_w, &L.i_w, &L.o2_w, &L.q_b, &L.k_b, &L.v_b, &L.o_b,
                                   &L.i_b, &L.o2_b, &L.ln_att_w, &L.ln_att_b, &L.ln_out_w, &L.ln_out_b};
        for (const HostTensor *t : all)
            if (!t->present()) { err = "missing tensor in encoder.layer." + std::to_string(l); return false; }
    }
    if (verbose)
        std::printf("bert_load_from_file: model size = %8.2f MB / num tensors = %d\n",
                    m.total_bytes / 1024.0 / 1024.0, m.n_tensors);
    return true;
}

// ---------------------------------------------------------------------------
// quantizer: same block rules as the reference's quantize tool (ggml
// quantize_row_q4_0/q4_1 reference forms; q8_0 per ggml quantize_row_q8_0).
// ---------------------------------------------------------------------------

static void quant_block(int itype, const float *x, uint8_t *o)
{
    if (itype == FMT_Q4_0) {
        float amax = 0.f, vmax = 0.f;
        for (int j = 0; j < 32; ++j)
            if (amax < std::fabs(x[j])) { amax = std::fabs(x[j]); vmax = x[j]; }
        const float d = vmax / -8, id = d != 0.f ? 1.0f / d : 0.0f;
        const uint16_t dh = f32_to_f16(d);
        std::memcpy(o, &dh, 2);
        for (int j = 0; j < 16; ++j) {
            int a = (int8_t)(x[j] * id + 8.5f), b = (int8_t)(x[j + 16] * id + 8.5f);
            a = a > 15 ? 15 : a; b = b > 15 ? 15 : b;
            o[2 + j] = (uint8_t)((uint8_t)a | ((uint8_t)b << 4));
        }
    } else if (itype == FMT_Q4_1) {
        float lo = 3.402823466e+38f, hi = -3.402823466e+38f;
        for (int j = 0; j < 32; ++j) { lo = x[j] < lo ? x[j] : lo; hi = x[j] > hi ? x[j] : hi; }
        const float d = (hi - lo) / 15, id = d != 0.f ? 1.0f / d : 0.0f;
        const uint16_t dh = f32_to_f16(d), mh = f32_to_f16(lo);
        std::memcpy(o, &dh, 2);
        std::memcpy(o + 2, &mh, 2);
        for (int j = 0; j < 16; ++j) {
            int a = (int8_t)((x[j] - lo) * id + 0.5f), b = (int8_t)((x[j + 16] - lo) * id + 0.5f);
            a = a > 15 ? 15 : a; b = b > 15 ? 15 : b;
            o[4 + j] = (uint8_t)((uint8_t)a | ((uint8_t)b << 4));
        }
    } else {  // q8_0
        float amax = 0.f;
        for (int j = 0; j < 32; ++j) amax = std::fmax(amax, std::fabs(x[j]));
        const float d = amax / 127, id = d != 0.f ? 1.0f / d : 0.0f;
        const uint16_t dh = f32_to_f16(d);
        std::memcpy(o, &dh, 2);
        for (int j = 0; j < 32; ++j) o[2 + j] = (uint8_t)(int8_t)std::roundf(x[j] * id);
    }
}

void quantize_row(int fmt, const float *x, uint8_t *dst, int64_t k)
{
    if (fmt == FMT_F32) { std::memcpy(dst, x, (size_t)k * 4); return; }
    if (fmt == FMT_F16) {
        for (int64_t i = 0; i < k; ++i) { const uint16_t h = f32_to_f16(x[i]); std::memcpy(dst + 2 * i, &h, 2); }
        return;
    }
    for (int64_t b = 0; b < k / QK; ++b) quant_block(fmt, x + QK * b, dst + fmt_block_bytes(fmt) * (size_t)b);
}

int quantize_file(const char *in, const char *out, int itype, bool verbose)
{
    if (itype != FMT_Q4_0 && itype != FMT_Q4_1 && itype != FMT_Q8_0) {
        errorf("bert_model_quantize: invalid quantization type %d\n", itype);
        return 1;
    }
    File fi(in, "rb");
    if (!fi.f) { errorf("bert_model_quantize: failed to open '%s' for reading\n", in); return 1; }
    File fo(out, "wb");
    if (!fo.f) { errorf("bert_model_quantize: failed to open '%s' for writing\n", out); return 1; }
    uint32_t magic = 0;
    int32_t hp[7];
    if (!fi.read(&magic, 4) || magic != 0x67676d6cu || !fi.read(hp, sizeof(hp))) {
        errorf("bert_model_quantize: invalid model file '%s' (bad magic)\n", in);
        return 1;
    }
    hp[6] = itype;
    fo.write(&magic, 4);
    fo.write(hp, sizeof(hp));
    std::vector<char> w;
    for (int i = 0; i < hp[0]; ++i) {
        uint32_t len;
        if (!fi.read(&len, 4)) return 1;
        w.resize(len);
        if (len && !fi.read(w.data(), len)) return 1;
        fo.write(&len, 4);
        if (len) fo.write(w.data(), len);
    }
    size_t org = 0, neu = 0;
    for (;;) {
        int32_t h3[3];
        if (!fi.read(h3, sizeof(h3))) break;
        int32_t ne[2] = {1, 1};
        if (h3[0] < 1 || h3[0] > 2 || !fi.read(ne, 4 * (size_t)h3[0]) || h3[1] <= 0 || h3[1] > 4096) return 1;
        std::string name((size_t)h3[1], '\0');
        if (!fi.read(&name[0], (size_t)h3[1])) return 1;
        const bool q = h3[0] == 2 && name.size() >= 6 && name.compare(name.size() - 6, 6, "weight") == 0;
        if (!fmt_valid(h3[2])) return 1;
        std::vector<uint8_t> src(fmt_row_bytes(h3[2], ne[0]) * (size_t)ne[1]);
        if (!fi.read(src.data(), src.size())) return 1;
        const int32_t oh[3] = {h3[0], h3[1], q ? itype : h3[2]};
        fo.write(oh, sizeof(oh));
        fo.write(ne, 4 * (size_t)h3[0]);
        fo.write(name.data(), name.size());
        org += (size_t)ne[0] * ne[1] * 4;
        if (q) {
            if (h3[2] != FMT_F32 && h3[2] != FMT_F16) {
                errorf("bert_model_quantize: unsupported ftype %d for integer quantization\n", h3[2]);
                return 1;
            }
            if (ne[0] % QK) { errorf("bert_model_quantize: row of '%s' not a multiple of 32\n", name.c_str()); return 1; }
            std::vector<float> row((size_t)ne[0]);
            std::vector<uint8_t> qrow(fmt_row_bytes(itype, ne[0]));
            const size_t rb = fmt_row_bytes(h3[2], ne[0]);
            for (int32_t r = 0; r < ne[1]; ++r) {
                dequant_row(h3[2], src.data() + rb * r, row.data(), ne[0]);
                for (int32_t b = 0; b < ne[0] / QK; ++b)
                    quant_block(itype, row.data() + b * QK, qrow.data() + fmt_block_bytes(itype) * b);
                fo.write(qrow.data(), qrow.size());
            }
            neu += qrow.size() * (size_t)ne[1];
            if (verbose) std::printf("%48s - [%5d, %5d] quantized\n", name.c_str(), ne[0], ne[1]);
        } else {
            fo.write(src.data(), src.size());
            neu += src.size();
        }
    }
    if (verbose) {
        std::printf("bert_model_quantize: model size  = %8.2f MB\n", org / 1024.0 / 1024.0);
        std::printf("bert_model_quantize: quant size  = %8.2f MB\n", neu / 1024.0 / 1024.0);
    }
    return 0;
}

}  // namespace emb
