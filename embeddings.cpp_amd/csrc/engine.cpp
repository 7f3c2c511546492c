// Per-GPU engine: weight repack + upload, workspace, forward launch sequence,
// live per-kernel timing.  See kernels.h for the HBM layouts.
#include "engine.h"

#include <algorithm>
#include <functional>
#include <map>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>

namespace emb {

#define HIP_OK(expr)                                                                                     \
    do {                                                                                                 \
        hipError_t e_ = (expr);                                                                          \
        if (e_ != hipSuccess) {                                                                          \
            errorf("libbert: HIP error %s at %s:%d (%s)\n", hipGetErrorString(e_), __FILE__, \
                         __LINE__, #expr);                                                               \
            return false;                                                                                \
        }                                                                                                \
    } while (0)

#define HIP_RC(expr)                                                                                     \
    do {                                                                                                 \
        hipError_t e_ = (expr);                                                                          \
        if (e_ != hipSuccess) {                                                                          \
            errorf("libbert: HIP error %s at %s:%d (%s)\n", hipGetErrorString(e_), __FILE__, \
                         __LINE__, #expr);                                                               \
            return -1;                                                                                   \
        }                                                                                                \
    } while (0)

const char *kclass_name(int k)
{
    static const char *names[K_NUM_CLASSES] = {"embed_ln", "gemm_qkv", "attention", "gemm_attn_out",
                                               "ln_stats", "gemm_ffn_up", "gemm_ffn_down", "pool_l2"};
    return (k >= 0 && k < K_NUM_CLASSES) ? names[k] : "?";
}

int hip_device_count()
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

namespace {

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// One host-side staged buffer of the replica.
struct Piece {
    std::vector<uint8_t> bytes;
    size_t off = 0;
};

void repack_linear(const std::vector<const HostTensor *> &parts, int fmt_dev, Piece &qs, Piece &dpl, Piece &mpl,
                   int &N_out, int &K_out);

// f32 weights (ftype 0 files, bert.cpp:499-503): each row w becomes the f16 pair
// hi = f16(w), lo = f16(w - hi) laid out as ONE f16 row of 2K, [hi | lo]; the GEMM
// reads X twice along that K (DevWeight::kx), so acc = X W_hi^T + X W_lo^T in f32
// with the weights good to ~2^-22 instead of f16's 2^-11.
void repack_linear_f32(const std::vector<const HostTensor *> &parts, Piece &qs, Piece &dpl, Piece &mpl, int &N_out,
                       int &K_out)
{
    const int K = parts[0]->ne0;
    std::vector<HostTensor> hl(parts.size());
    std::vector<const HostTensor *> hp;
    for (size_t i = 0; i < parts.size(); ++i) {
        const HostTensor &t = *parts[i];
        HostTensor &o = hl[i];
        o.fmt = FMT_F16; o.ne0 = 2 * K; o.ne1 = t.ne1;
        o.bytes.assign((size_t)t.ne1 * 2 * K * 2, 0);
        std::vector<float> row((size_t)K);
        for (int r = 0; r < t.ne1; ++r) {
            dequant_row(t.fmt, t.bytes.data() + fmt_row_bytes(t.fmt, K) * r, row.data(), K);
            uint16_t *dst = (uint16_t *)o.bytes.data() + (size_t)r * 2 * K;
            for (int k = 0; k < K; ++k) {
                const uint16_t h = f32_to_f16(row[(size_t)k]);
                dst[k] = h;
                dst[K + k] = f32_to_f16(row[(size_t)k] - f16_to_f32(h));
            }
        }
        hp.push_back(&o);
    }
    repack_linear(hp, FMT_F16, qs, dpl, mpl, N_out, K_out);
}

// Linear weight [N][K] (file rows) -> the lane-order device layout (kernels.h).
void repack_linear(const std::vector<const HostTensor *> &parts, int fmt_dev, Piece &qs, Piece &dpl, Piece &mpl,
                   int &N_out, int &K_out)
{
    if (fmt_dev == FMT_F32) {
        repack_linear_f32(parts, qs, dpl, mpl, N_out, K_out);
        return;
    }
    const int K = parts[0]->ne0;
    int N = 0;
    for (const HostTensor *t : parts) N += t->ne1;
    N_out = N;
    K_out = K;
    const size_t G = (size_t)N / 32;
    const size_t QB = fmt_dev == FMT_F16 ? 64 : fmt_dev == FMT_Q8_0 ? 32 : 16;
    qs.bytes.assign((size_t)(K / 64) * G * 64 * QB, 0);
    if (fmt_dev != FMT_F16) dpl.bytes.assign((size_t)N * (K / 32) * 2, 0);
    if (fmt_dev == FMT_Q4_1) mpl.bytes.assign((size_t)N * (K / 32) * 2, 0);
    uint16_t *dd = (uint16_t *)dpl.bytes.data();
    uint16_t *mm = fmt_dev == FMT_Q4_1 ? (uint16_t *)mpl.bytes.data() : nullptr;
    static const int pos4[4] = {0, 2, 1, 3};
    int n = 0;
    for (const HostTensor *t : parts) {
        const size_t rb = fmt_row_bytes(t->fmt, K), bb = fmt_block_bytes(t->fmt);
        for (int r = 0; r < t->ne1; ++r, ++n) {
            const uint8_t *src = t->bytes.data() + rb * r;
            const size_t grp = (size_t)n / 32;
            const int a = (n % 32) / 16, f = n % 16;
            for (int blk = 0; blk < K / 32; ++blk) {
                const size_t ks = (size_t)blk / 2;
                const int u = 2 * a + (blk & 1);
                const size_t rec0 = (ks * G + grp) * 64;            // lane-record index of lane 0
                const size_t di = ((ks * G + grp) * 16 + f) * 4 + u;
                for (int e = 0; e < 32; ++e) {
                    const int g = e / 8, i = e % 8;
                    uint8_t *o = qs.bytes.data() + (rec0 + 16 * g + f) * QB;
                    const int k = 32 * blk + e;
                    if (fmt_dev == FMT_F16) {
                        uint16_t h;
                        if (t->fmt == FMT_F16) std::memcpy(&h, src + 2 * k, 2);
                        else { float v; std::memcpy(&v, src + 4 * k, 4); h = f32_to_f16(v); }
                        std::memcpy(o + 16 * u + 2 * i, &h, 2);
                    } else if (fmt_dev == FMT_Q8_0) {
                        const int8_t q = (int8_t)src[bb * blk + 2 + e];
                        o[8 * u + 4 * (i / 4) + pos4[i % 4]] = (uint8_t)((uint8_t)q ^ 0x80u);
                    } else {
                        const uint8_t *nib = src + bb * blk + (fmt_dev == FMT_Q4_1 ? 4 : 2);
                        const uint32_t q = e < 16 ? (nib[e] & 15u) : (uint32_t)(nib[e - 16] >> 4);
                        uint32_t w;
                        std::memcpy(&w, o + 4 * u, 4);
                        w |= q << (4 * (i / 2) + 16 * (i % 2));
                        std::memcpy(o + 4 * u, &w, 4);
                    }
                }
                if (fmt_dev != FMT_F16) std::memcpy(&dd[di], src + bb * blk, 2);
                if (mm) std::memcpy(&mm[di], src + bb * blk + 2, 2);
            }
        }
    }
}

// LN fold constants (kernels.h) of a projection W (the concatenated parts) that
// reads LN(y) = gamma (y - mean) r + beta: c1[n] = sum_k W[n][k] gamma[k],
// c2[n] = b[n] + sum_k W[n][k] beta[k], with W as the GEMM multiplies it (each
// weight rounded once to f16 after dequantization, or the f32 value itself for
// the hi/lo pairs of f32 files), summed in double.
void fold_ln(const std::vector<const HostTensor *> &parts, const std::vector<const HostTensor *> &bias,
             const HostTensor &gamma, const HostTensor &beta, Piece &c1, Piece &c2, bool exact)
{
    const int K = parts[0]->ne0;
    const float *gm = (const float *)gamma.bytes.data(), *bt = (const float *)beta.bytes.data();
    std::vector<float> row((size_t)K), o1, o2;
    for (const HostTensor *t : parts) {
        const size_t rb = fmt_row_bytes(t->fmt, K);
        for (int r = 0; r < t->ne1; ++r) {
            dequant_row(t->fmt, t->bytes.data() + rb * r, row.data(), K);
            double s1 = 0.0, s2 = 0.0;
            for (int k = 0; k < K; ++k) {
                // the weight as the GEMM multiplies it: f16-rounded, or hi + lo (f32 files)
                const double w = exact ? (double)row[(size_t)k] : (double)f16_to_f32(f32_to_f16(row[(size_t)k]));
                s1 += w * gm[k];
                s2 += w * bt[k];
            }
            o1.push_back((float)s1);
            o2.push_back((float)s2);
        }
    }
    size_t n = 0;
    for (const HostTensor *b : bias) {
        const float *bv = (const float *)b->bytes.data();
        for (int i = 0; i < b->ne0; ++i, ++n) o2[n] = (float)((double)o2[n] + (double)bv[i]);
    }
    c1.bytes.assign((const uint8_t *)o1.data(), (const uint8_t *)(o1.data() + o1.size()));
    c2.bytes.assign((const uint8_t *)o2.data(), (const uint8_t *)(o2.data() + o2.size()));
}

// Embedding table in its file format -> aligned planes.
void repack_table(const HostTensor &t, Piece &qs, Piece &dpl, Piece &mpl)
{
    const int rows = t.ne1, cols = t.ne0;
    if (t.fmt == FMT_F32 || t.fmt == FMT_F16) {
        qs.bytes = t.bytes;
        return;
    }
    const size_t nblk = (size_t)rows * (cols / 32), bb = fmt_block_bytes(t.fmt);
    const size_t qb = t.fmt == FMT_Q8_0 ? 32 : 16;
    qs.bytes.assign(nblk * qb, 0);
    dpl.bytes.assign(nblk * 2, 0);
    if (t.fmt == FMT_Q4_1) mpl.bytes.assign(nblk * 2, 0);
    for (size_t i = 0; i < nblk; ++i) {
        const uint8_t *blk = t.bytes.data() + i * bb;
        std::memcpy(dpl.bytes.data() + 2 * i, blk, 2);
        if (t.fmt == FMT_Q4_1) {
            std::memcpy(mpl.bytes.data() + 2 * i, blk + 2, 2);
            std::memcpy(qs.bytes.data() + 16 * i, blk + 4, 16);
        } else {
            std::memcpy(qs.bytes.data() + qb * i, blk + 2, qb);
        }
    }
}

}  // namespace

ModelImage::~ModelImage()
{
    if (pinned_) (void)hipHostFree(pinned_);
}

bool build_model_image(const HostModel &m, ModelImage &img, std::string &err, bool pin)
{
    try {
        const HParams &hp = m.hp;
        const int d = hp.n_embd, f = hp.n_intermediate;
        if (hp.n_head <= 0 || d % 64 || d > 1024 || f % 64 || (d / hp.n_head != 32 && d / hp.n_head != 64)) {
            char buf[256];
            std::snprintf(buf, sizeof buf,
                          "unsupported shape n_embd=%d n_intermediate=%d n_head=%d (need n_embd %% 64 == 0, "
                          "n_embd <= 1024, head_dim 32 or 64)", d, f, hp.n_head);
            err = buf;
            return false;
        }
        if (fault_inject("image")) throw std::bad_alloc();
        img.hp = hp;
        img.wfmt = hp.ftype;
        // f32 files run the f32 chain (f32.hip) on the file's own f32 rows; the other
        // formats the lane-order layout of the MFMA f16 GEMMs
        img.f32 = img.wfmt == FMT_F32;
        std::vector<Piece> pieces;
        pieces.reserve(16 + 24 * (size_t)hp.n_layer);
        auto add = [&](Piece &&p) -> size_t { pieces.push_back(std::move(p)); return pieces.size() - 1; };
        auto vec = [&](const HostTensor &t) -> size_t { Piece p; p.bytes = t.bytes; return add(std::move(p)); };
        auto table = [&](const HostTensor &t) -> ModelImage::Tab {
            Piece q, dd, mm;
            repack_table(t, q, dd, mm);
            ModelImage::Tab r;
            r.fmt = t.fmt; r.rows = t.ne1; r.cols = t.ne0;
            r.q = add(std::move(q)); r.d = add(std::move(dd)); r.m = add(std::move(mm));
            return r;
        };
        auto linear = [&](std::vector<const HostTensor *> parts) -> ModelImage::Lin {
            Piece q, dd, mm;
            ModelImage::Lin r;
            repack_linear(parts, img.wfmt, q, dd, mm, r.N, r.K);
            r.q = add(std::move(q)); r.d = add(std::move(dd)); r.m = add(std::move(mm));
            return r;
        };
        img.word = table(m.word);
        img.type = table(m.ttype);
        img.pos = table(m.pos);
        // f32 chain: the era's fp16 GELU and exp tables, built on the host (libm) as
        // ggml built them, indexed on the device by the f16 bits of the input
        if (img.f32) {
            std::vector<uint16_t> tg, te;
            era_tables(tg, te);
            Piece pg, pe;
            pg.bytes.assign((const uint8_t *)tg.data(), (const uint8_t *)(tg.data() + tg.size()));
            pe.bytes.assign((const uint8_t *)te.data(), (const uint8_t *)(te.data() + te.size()));
            img.gelu = add(std::move(pg));
            img.exp = add(std::move(pe));
        }
        img.lnw = vec(m.ln_e_w);
        img.lnb = vec(m.ln_e_b);
        auto fold = [&](std::vector<const HostTensor *> parts, std::vector<const HostTensor *> bias,
                        const HostTensor &gamma, const HostTensor &beta, size_t &i1, size_t &i2) {
            Piece c1, c2;
            fold_ln(parts, bias, gamma, beta, c1, c2, img.wfmt == FMT_F32);
            i1 = add(std::move(c1));
            i2 = add(std::move(c2));
        };
        // f32 chain: the rows of the parts as f32 (concatenated along N)
        auto rows32 = [&](std::vector<const HostTensor *> parts) -> size_t {
            Piece p;
            for (const HostTensor *t : parts) {
                const size_t n0 = p.bytes.size();
                p.bytes.resize(n0 + (size_t)t->ne1 * t->ne0 * 4);
                for (int r = 0; r < t->ne1; ++r)
                    dequant_row(t->fmt, t->bytes.data() + fmt_row_bytes(t->fmt, t->ne0) * r,
                                (float *)(p.bytes.data() + n0) + (size_t)r * t->ne0, t->ne0);
            }
            return add(std::move(p));
        };
        img.layers.assign((size_t)hp.n_layer, ModelImage::Layer());
        for (int l = 0; l < hp.n_layer; ++l) {
            const HostLayer &L = m.layers[(size_t)l];
            ModelImage::Layer &x = img.layers[(size_t)l];
            if (img.f32) {
                x.w32q = rows32({&L.q_w, &L.k_w, &L.v_w}); x.w32o = rows32({&L.o_w});
                x.w32u = rows32({&L.i_w}); x.w32d = rows32({&L.o2_w});
                x.bq = rows32({&L.q_b, &L.k_b, &L.v_b}); x.bu = vec(L.i_b);
                x.bo = vec(L.o_b); x.bdown = vec(L.o2_b);
                x.l1w = vec(L.ln_att_w); x.l1b = vec(L.ln_att_b); x.l2w = vec(L.ln_out_w); x.l2b = vec(L.ln_out_b);
                continue;
            }
            x.qkv = linear({&L.q_w, &L.k_w, &L.v_w});
            x.o = linear({&L.o_w});
            x.up = linear({&L.i_w});
            x.down = linear({&L.o2_w});
            // the LN in front of QKV: the previous layer's output LN, or the embedding LN
            const HostTensor &gq = l ? m.layers[(size_t)l - 1].ln_out_w : m.ln_e_w;
            const HostTensor &bq = l ? m.layers[(size_t)l - 1].ln_out_b : m.ln_e_b;
            fold({&L.q_w, &L.k_w, &L.v_w}, {&L.q_b, &L.k_b, &L.v_b}, gq, bq, x.c1q, x.c2q);
            fold({&L.i_w}, {&L.i_b}, L.ln_att_w, L.ln_att_b, x.c1u, x.c2u);
            x.bo = vec(L.o_b); x.bdown = vec(L.o2_b);
            x.l1w = vec(L.ln_att_w); x.l1b = vec(L.ln_att_b); x.l2w = vec(L.ln_out_w); x.l2b = vec(L.ln_out_b);
        }
        img.off.resize(pieces.size());
        img.len.resize(pieces.size());
        size_t total = 0;
        for (size_t i = 0; i < pieces.size(); ++i) {
            img.off[i] = total;
            img.len[i] = pieces[i].bytes.size();
            total += align_up(pieces[i].bytes.size(), 256);
        }
        img.total = total ? total : 256;
        // one contiguous image, page-locked when possible so each replica's upload is
        // one async copy on its own stream; pieces are freed as they are copied
        uint8_t *dst = nullptr;
        if (pin) {
            if (hipHostMalloc((void **)&img.pinned_, img.total, hipHostMallocPortable) != hipSuccess) {   // every device copies from it
                (void)hipGetLastError();
                img.pinned_ = nullptr;
                trace("build_model_image: page-locking %zu bytes failed, pageable uploads\n", img.total);
            }
        }
        if (img.pinned_) {
            dst = img.pinned_;
        } else {
            img.host_.assign(img.total, 0);
            dst = img.host_.data();
        }
        for (size_t i = 0; i < pieces.size(); ++i) {
            Piece &p = pieces[i];
            if (!p.bytes.empty()) std::memcpy(dst + img.off[i], p.bytes.data(), p.bytes.size());
            const size_t pad = align_up(p.bytes.size(), 256) - p.bytes.size();
            if (pad) std::memset(dst + img.off[i] + p.bytes.size(), 0, pad);
            std::vector<uint8_t>().swap(p.bytes);
        }
        return true;
    } catch (const std::bad_alloc &) {
        err = "out of host memory building the device image";
    } catch (const std::exception &ex) {
        err = std::string("building the device image failed: ") + ex.what();
    }
    return false;
}

Device::Device(int ordinal, const ModelImage &img) : ordinal_(ordinal), hp_(img.hp)
{
    DeviceGuard g(ordinal);
    if (!g.ok() || hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&done_ev_, hipEventDisableTiming) != hipSuccess) {
        (void)hipGetLastError();
        errorf("libbert: cannot initialise HIP device %d\n", ordinal);
        return;
    }
    if (hipMalloc((void **)&arena_, img.total) != hipSuccess) {
        (void)hipGetLastError();
        errorf("libbert: hipMalloc of %zu bytes of weights failed on device %d\n", img.total, ordinal_);
        arena_ = nullptr;
        return;
    }
    arena_size_ = img.total;
    // page-locked image: one async copy on this replica's stream, so the uploads of
    // all replicas overlap although one thread issues them; pageable: a blocking copy
    const hipError_t e = img.pinned()
        ? hipMemcpyAsync(arena_, img.bytes(), img.total, hipMemcpyHostToDevice, stream_)
        : hipMemcpy(arena_, img.bytes(), img.total, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        errorf("libbert: weight upload failed on device %d: %s\n", ordinal_, hipGetErrorString(e));
        return;
    }
    bind(img);
    uploading_ = true;
}

bool Device::finish_load()
{
    if (!uploading_) return false;
    DeviceGuard g(ordinal_);
    if (!g.ok()) return false;
    const hipError_t e = hipStreamSynchronize(stream_);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        errorf("libbert: weight upload failed on device %d: %s\n", ordinal_, hipGetErrorString(e));
        return false;
    }
    uploading_ = false;
    ok_ = true;
    return true;
}

Device::~Device()
{
    DeviceGuard g(ordinal_);
    if (stream_ && uploading_) (void)hipStreamSynchronize(stream_);   // the image may still be in flight
    if (done_ev_ && any_forward_) (void)hipEventSynchronize(done_ev_);
    if (stream_) (void)hipStreamSynchronize(stream_);
    drop_graphs();
    for (auto &p : pending_) { (void)hipEventDestroy(p.a); (void)hipEventDestroy(p.b); }
    for (auto e : free_events_) (void)hipEventDestroy(e);
    if (arena_) (void)hipFree(arena_);
    if (ws_) (void)hipFree(ws_);
    if (h_ids_) (void)hipHostFree(h_ids_);
    if (h_cu_) (void)hipHostFree(h_cu_);
    if (h_out_) (void)hipHostFree(h_out_);
    if (done_ev_) (void)hipEventDestroy(done_ev_);
    if (stream_) (void)hipStreamDestroy(stream_);
}

void Device::order_after_last(hipStream_t s)
{
    if (any_forward_ && last_stream_ != s) (void)hipStreamWaitEvent(s, done_ev_, 0);
}

void Device::mark_done(hipStream_t s)
{
    (void)hipEventRecord(done_ev_, s);
    last_stream_ = s;
    any_forward_ = true;
}

void Device::bind(const ModelImage &img)
{
    wfmt_ = img.wfmt;
    f32_ = img.f32;
    auto P = [&](size_t i) -> void * {
        return (i == ModelImage::kNone || img.len[i] == 0) ? nullptr : (void *)(arena_ + img.off[i]);
    };
    auto mk_table = [&](const ModelImage::Tab &x) {
        DevTable r;
        r.fmt = x.fmt; r.rows = x.rows; r.cols = x.cols;
        r.qs = P(x.q); r.d = (const uint16_t *)P(x.d); r.m = (const uint16_t *)P(x.m);
        return r;
    };
    if (f32_) {
        gelu_tab_ = (const uint16_t *)P(img.gelu);
        exp_tab_ = (const uint16_t *)P(img.exp);
    }
    word_ = mk_table(img.word);
    type_ = mk_table(img.type);
    pos_ = mk_table(img.pos);
    ln_e_w_ = (float *)P(img.lnw);
    ln_e_b_ = (float *)P(img.lnb);
    auto mk_lin = [&](const ModelImage::Lin &x) {
        DevWeight w;
        w.fmt = wfmt_ == FMT_F32 ? FMT_F16 : wfmt_; w.N = x.N; w.K = x.K;
        w.kx = wfmt_ == FMT_F32 ? x.K / 2 : 0;
        w.qs = P(x.q); w.d = (const uint16_t *)P(x.d); w.m = (const uint16_t *)P(x.m);
        return w;
    };
    layers_.assign((size_t)hp_.n_layer, DevLayer());
    for (int l = 0; l < hp_.n_layer; ++l) {
        const ModelImage::Layer &x = img.layers[(size_t)l];
        DevLayer &D = layers_[(size_t)l];
        if (f32_) {
            D.w32_qkv = (const float *)P(x.w32q); D.w32_o = (const float *)P(x.w32o);
            D.w32_up = (const float *)P(x.w32u); D.w32_down = (const float *)P(x.w32d);
            D.b_qkv = (const float *)P(x.bq); D.b_up = (const float *)P(x.bu);
            D.b_o = (float *)P(x.bo); D.b_down = (float *)P(x.bdown);
            D.ln1_w = (float *)P(x.l1w); D.ln1_b = (float *)P(x.l1b); D.ln2_w = (float *)P(x.l2w); D.ln2_b = (float *)P(x.l2b);
            continue;
        }
        D.qkv = mk_lin(x.qkv); D.o = mk_lin(x.o); D.up = mk_lin(x.up); D.down = mk_lin(x.down);
        D.b_o = (float *)P(x.bo); D.b_down = (float *)P(x.bdown);
        D.c1_qkv = (float *)P(x.c1q); D.c2_qkv = (float *)P(x.c2q); D.c1_up = (float *)P(x.c1u); D.c2_up = (float *)P(x.c2u);
        D.ln1_w = (float *)P(x.l1w); D.ln1_b = (float *)P(x.l1b); D.ln2_w = (float *)P(x.l2w); D.ln2_b = (float *)P(x.l2b);
    }
}

bool Device::reserve(int64_t tokens, int64_t seqs, int max_len)
{
    const int64_t pool_rows = seqs * pool_chunks(std::max(1, std::min(max_len, hp_.n_max_tokens)));
    if (tokens <= cap_tokens_ && seqs <= cap_seqs_ && pool_rows <= cap_pool_) return true;
    DeviceGuard g(ordinal_);
    HIP_OK(g.status());
    if (any_forward_) HIP_OK(hipEventSynchronize(done_ev_));   // the last forward may be on a caller stream
    HIP_OK(hipStreamSynchronize(stream_));
    const int64_t nt = std::max<int64_t>(align_up((size_t)std::max(tokens, cap_tokens_), 4096), 4096);
    const int64_t ns = std::max<int64_t>(align_up((size_t)std::max(seqs, cap_seqs_), 256), 256);
    // pool partials [n_seqs][chunks][d]: sized by the sentences' own max_len, not
    // n_max_tokens (a chunk of many short texts would otherwise reserve GBs)
    const int64_t np = std::max<int64_t>(align_up((size_t)std::max(pool_rows, cap_pool_), 256), 256);
    const int64_t rows = nt + GEMM_BM + 256;   // padding rows for tile overrun (kernels read, never trust)
    const int64_t d = hp_.n_embd, f = hp_.n_intermediate;
    size_t off = 0;
    auto take = [&](size_t bytes) { size_t o = off; off += align_up(bytes, 256); return o; };
    // f16 chain: Z, QKV, ATT, FFN f16 + statistics; f32 chain: X, Z, QKV, ATT, FFN f32
    const int64_t r16 = f32_ ? 0 : rows, r32 = f32_ ? rows : 0;
    const size_t o_st = take(r16 * 8), o_z = take(r16 * d * 2), o_part = take(r16 * (d / 32) * 8);
    const size_t o_qkv = take(r16 * 3 * d * 2), o_att = take(r16 * d * 2), o_ffn = take(r16 * f * 2);
    const size_t o_x32 = take(r32 * d * 4), o_z32 = take(r32 * d * 4), o_qkv32 = take(r32 * 3 * d * 4);
    const size_t o_att32 = take(r32 * d * 4), o_ffn32 = take(r32 * f * 4);
    const size_t o_ids = take(rows * 4), o_cu = take((ns + 1) * 4), o_out = take(ns * d * 4);
    const size_t o_pool = take((size_t)np * d * 4);
    drop_graphs();   // captured graphs hold the old workspace pointers
    if (ws_) { (void)hipFree(ws_); ws_ = nullptr; }
    if (h_ids_) { (void)hipHostFree(h_ids_); h_ids_ = nullptr; }
    if (h_cu_) { (void)hipHostFree(h_cu_); h_cu_ = nullptr; }
    if (h_out_) { (void)hipHostFree(h_out_); h_out_ = nullptr; }
    cap_tokens_ = cap_seqs_ = cap_pool_ = 0;
    HIP_OK(hipMalloc((void **)&ws_, off));
    // on the replica's own (non-blocking) stream: a null-stream memset would not
    // be ordered before the forward that follows on stream_
    HIP_OK(hipMemsetAsync(ws_, 0, off, stream_));
    HIP_OK(hipStreamSynchronize(stream_));
    st_ = (float2 *)(ws_ + o_st); z_ = (uint16_t *)(ws_ + o_z); part_ = (float2 *)(ws_ + o_part);
    rows_ = rows;
    qkv_ = (uint16_t *)(ws_ + o_qkv); att_ = (uint16_t *)(ws_ + o_att); ffn_ = (uint16_t *)(ws_ + o_ffn);
    d_ids_ = (int32_t *)(ws_ + o_ids); d_cu_ = (int32_t *)(ws_ + o_cu); d_out_ = (float *)(ws_ + o_out);
    pool_part_ = (float *)(ws_ + o_pool);
    x32_ = (float *)(ws_ + o_x32); z32_ = (float *)(ws_ + o_z32); qkv32_ = (float *)(ws_ + o_qkv32);
    att32_ = (float *)(ws_ + o_att32); ffn32_ = (float *)(ws_ + o_ffn32);
    HIP_OK(hipHostMalloc((void **)&h_ids_, nt * 4, hipHostMallocDefault));
    HIP_OK(hipHostMalloc((void **)&h_cu_, (ns + 1) * 4, hipHostMallocDefault));
    HIP_OK(hipHostMalloc((void **)&h_out_, ns * d * 4, hipHostMallocDefault));
    cap_tokens_ = nt;
    cap_seqs_ = ns;
    cap_pool_ = np;
    return true;
}

hipEvent_t Device::get_event()
{
    if (!free_events_.empty()) { hipEvent_t e = free_events_.back(); free_events_.pop_back(); return e; }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
}

void Device::begin(int cls, hipStream_t s, hipEvent_t &a)
{
    (void)cls;
    a = nullptr;
    if (!profiling_) return;
    a = get_event();
    (void)hipEventRecord(a, s);
}

void Device::end(int cls, hipStream_t s, hipEvent_t a, double work)
{
    if (!profiling_ || !a) return;
    hipEvent_t b = get_event();
    (void)hipEventRecord(b, s);
    pending_.push_back({cls, a, b, work});
}

void Device::collect_stats()
{
    DeviceGuard g(ordinal_);
    for (auto &p : pending_) {
        (void)hipEventSynchronize(p.b);
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            stats_[p.cls].launches += 1;
            stats_[p.cls].ms += ms;
            stats_[p.cls].work += p.work;
        }
        free_events_.push_back(p.a);
        free_events_.push_back(p.b);
    }
    pending_.clear();
}

void Device::reset_stats()
{
    collect_stats();
    for (auto &s : stats_) s = KStats();
}

void Device::drop_graphs()
{
    for (auto &g : graphs_) (void)hipGraphExecDestroy(g.exec);
    graphs_.clear();
    seen_once_.clear();
}

int Device::forward(const int32_t *d_ids, const int32_t *d_cu, int n_seqs, int max_len, int T, float *d_out,
                    hipStream_t s, double len2_sum)
{
    // attention work for the per-kernel stats: exact from the host's lengths when
    // known, else T max_len (exact for equal lengths, an upper bound otherwise)
    att_flop_ = 4.0 * hp_.n_embd * (len2_sum >= 0 ? len2_sum : (double)T * max_len);
    if (!ok_) return -3;
    if (T > cap_tokens_ || n_seqs > cap_seqs_ || (int64_t)n_seqs * pool_chunks(max_len) > cap_pool_) return -2;
    if (T <= 0 || n_seqs <= 0) return 0;
    order_after_last(s);
    const int rc = forward_ordered(d_ids, d_cu, n_seqs, max_len, T, d_out, s);
    mark_done(s);
    return rc;
}

int Device::forward_ordered(const int32_t *d_ids, const int32_t *d_cu, int n_seqs, int max_len, int T, float *d_out,
                            hipStream_t s)
{
    // BERT_CHECK_FINITE=1: after every kernel, count non-finite outputs over the
    // valid rows and report the first kernel that produced any (diagnostics).
    static const bool check = [] { const char *e = std::getenv("BERT_CHECK_FINITE"); return e && *e == '1'; }();
    static const bool graphs_env = [] { const char *e = std::getenv("BERT_GRAPHS"); return !(e && *e == '0'); }();
    if (profiling_ || check || !use_graphs_ || !graphs_env || s == nullptr)
        return launch_all(d_ids, d_cu, n_seqs, max_len, T, d_out, s, check);
    const GraphKey key{d_ids, d_cu, d_out, s, n_seqs, max_len, T};
    for (auto &g : graphs_)
        if (g.key == key) return hipGraphLaunch(g.exec, s) == hipSuccess ? 0 : -1;
    // a shape seen for the first time runs eagerly (one-off batches never pay
    // for a capture); on its second use the sequence is captured and replayed
    bool seen = false;
    for (auto &k : seen_once_) seen = seen || (k == key);
    if (!seen) {
        if (seen_once_.size() >= 32) seen_once_.erase(seen_once_.begin());
        seen_once_.push_back(key);
        return launch_all(d_ids, d_cu, n_seqs, max_len, T, d_out, s, false);
    }
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    if (hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) != hipSuccess) {
        (void)hipGetLastError();
        use_graphs_ = false;   // this runtime / stream cannot capture: stay eager
        return launch_all(d_ids, d_cu, n_seqs, max_len, T, d_out, s, false);
    }
    const int rc = launch_all(d_ids, d_cu, n_seqs, max_len, T, d_out, s, false);
    const hipError_t ec = hipStreamEndCapture(s, &graph);
    if (rc != 0 || ec != hipSuccess || hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0) != hipSuccess) {
        (void)hipGetLastError();
        if (graph) (void)hipGraphDestroy(graph);
        use_graphs_ = false;
        return launch_all(d_ids, d_cu, n_seqs, max_len, T, d_out, s, false);
    }
    (void)hipGraphDestroy(graph);
    if (graphs_.size() >= 8) {
        (void)hipGraphExecDestroy(graphs_.front().exec);
        graphs_.erase(graphs_.begin());
    }
    graphs_.push_back({key, exec});
    return hipGraphLaunch(exec, s) == hipSuccess ? 0 : -1;
}

int Device::launch_all(const int32_t *d_ids, const int32_t *d_cu, int n_seqs, int max_len, int T, float *d_out,
                       hipStream_t s, bool check)
{
    if (f32_) return launch_all_f32(d_ids, d_cu, n_seqs, max_len, T, d_out, s);
    const int d = hp_.n_embd, f = hp_.n_intermediate;
    const int M = gemm_rows(T);   // GEMM rows: T padded to whole tiles
    const double t = (double)T;
    hipEvent_t ev;
    unsigned *cnt = nullptr;
    bool bad = false;
    if (check) (void)hipMalloc((void **)&cnt, sizeof(unsigned));
    auto chk = [&](const char *what, int layer, const void *p, size_t n, int f16) {
        if (!check || bad) return;
        (void)hipMemsetAsync(cnt, 0, sizeof(unsigned), s);
        launch_count_nonfinite(p, n, f16, cnt, s);
        unsigned h = 0;
        (void)hipMemcpyAsync(&h, cnt, sizeof(unsigned), hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
        if (h) {
            bad = true;
            errorf("libbert: BERT_CHECK_FINITE: %u non-finite values after %s (layer %d)\n", h, what, layer);
        }
    };

    begin(K_EMBED_LN, s, ev);
    launch_embed_ln(word_, type_, pos_, ln_e_w_, d_ids, d_cu, n_seqs, max_len, d, z_, st_, s);
    end(K_EMBED_LN, s, ev, t * (4.0 + 3.0 * d * 2.0 + 2.0 * d + 8.0));
    chk("embed_ln", -1, z_, (size_t)T * d, 1);
    // z_ holds the stream as z = y * gamma of the LN in front of the next
    // projection, st_ its (mean, 1/sigma) (kernels.h LN fold); (gz, bz) is that LN
    const float *gz = ln_e_w_, *bz = ln_e_b_;
    const int G = d / 32;
    // Small batches: the projections combine their input's LN statistics from the
    // residual GEMM's partials themselves (LnFold::in_part; the column-0 tiles store
    // them for the residual GEMM after), so only the last ln_stats launch (for the
    // pool) remains: 2 n_layer - 1 fewer launches, the same bits (the combine is
    // ln_stats_kernel's arithmetic).  Where the tile config has no LDS for it (the
    // large-batch tiles, d > 768 on 64-row tiles), the statistics launches stay.
    static const bool fold_env = [] { const char *e = std::getenv("BERT_STATS_FOLD"); return !(e && *e == '0'); }();
    const bool fold = fold_env && !layers_.empty() && gemm_fold_ok(layers_[0].qkv, M, G) && gemm_fold_ok(layers_[0].up, M, G);

    const double att_flop = att_flop_;   // sum over sentences of 4 d len^2 (QK^T and PV), set by the caller
    for (int l = 0; l < hp_.n_layer; ++l) {
        const DevLayer &L = layers_[(size_t)l];
        LnFold in;
        if (fold && l > 0) {
            // the stream of the previous FFN-down: its partials; the rows' statistics
            // go to st_ for this layer's O-proj residual
            in.in_part = part_; in.in_part_stride = (int32_t)rows_; in.in_G = G; in.st_out = st_;
        } else {
            in.in_stats = st_;
        }
        in.c1 = L.c1_qkv;
        begin(K_GEMM_QKV, s, ev);
        if (launch_gemm(L.qkv, z_, M, L.c2_qkv, EPI_BIAS_F16, nullptr, qkv_, s, in) != 0) return -1;
        end(K_GEMM_QKV, s, ev, 2.0 * t * 3.0 * d * d);
        chk("gemm_qkv", l, qkv_, (size_t)T * 3 * d, 1);

        begin(K_ATTENTION, s, ev);
        launch_attention(qkv_, d_cu, n_seqs, max_len, hp_.n_head, d, att_, s);
        end(K_ATTENTION, s, ev, att_flop);
        chk("attention", l, att_, (size_t)T * d, 1);

        // y1 = LN(y) + ATT W_o^T + b_o, stored as z = y1 * gamma_1 with its partials
        LnFold r1;
        r1.res_stats = st_; r1.res_g = gz; r1.res_b = bz;
        r1.g_next = L.ln1_w; r1.part = part_; r1.part_stride = (int32_t)rows_;
        begin(K_GEMM_O, s, ev);
        if (launch_gemm(L.o, att_, M, L.b_o, EPI_BIAS_RES, z_, z_, s, r1) != 0) return -1;   // refused: z_ would be stale
        end(K_GEMM_O, s, ev, 2.0 * t * d * d);
        chk("gemm_o", l, z_, (size_t)T * d, 1);

        if (!fold) {
            begin(K_LN_STATS, s, ev);
            if (launch_ln_stats(part_, G, (int32_t)rows_, M, d, st_, s) != 0) return -1;
            end(K_LN_STATS, s, ev, (double)M * (G + 1) * 8.0);
        }
        gz = L.ln1_w; bz = L.ln1_b;

        if (fold) {
            in.in_stats = nullptr;
            in.in_part = part_; in.in_part_stride = (int32_t)rows_; in.in_G = G; in.st_out = st_;
        }
        in.c1 = L.c1_up;
        begin(K_GEMM_FFN_UP, s, ev);
        if (launch_gemm(L.up, z_, M, L.c2_up, EPI_BIAS_GELU_F16, nullptr, ffn_, s, in) != 0) return -1;
        end(K_GEMM_FFN_UP, s, ev, 2.0 * t * d * f);
        chk("gemm_up", l, ffn_, (size_t)T * f, 1);

        LnFold r2;
        r2.res_stats = st_; r2.res_g = gz; r2.res_b = bz;
        r2.g_next = L.ln2_w; r2.part = part_; r2.part_stride = (int32_t)rows_;
        begin(K_GEMM_FFN_DOWN, s, ev);
        if (launch_gemm(L.down, ffn_, M, L.b_down, EPI_BIAS_RES, z_, z_, s, r2) != 0) return -1;
        end(K_GEMM_FFN_DOWN, s, ev, 2.0 * t * d * f);
        chk("gemm_down", l, z_, (size_t)T * d, 1);

        if (!fold || l + 1 == hp_.n_layer) {   // (fold: only the pool's statistics)
            begin(K_LN_STATS, s, ev);
            if (launch_ln_stats(part_, G, (int32_t)rows_, M, d, st_, s) != 0) return -1;
            end(K_LN_STATS, s, ev, (double)M * (G + 1) * 8.0);
        }
        gz = L.ln2_w; bz = L.ln2_b;
    }
    begin(K_POOL_L2, s, ev);
    launch_pool_l2(z_, st_, gz, bz, d_cu, n_seqs, max_len, d, pool_part_, d_out, s);
    end(K_POOL_L2, s, ev, t * d * 2.0 + t * 8.0 + (double)n_seqs * d * 4.0);
    chk("pool_l2", -1, d_out, (size_t)n_seqs * d, 0);
    if (cnt) (void)hipFree(cnt);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        errorf("libbert: kernel launch failed: %s\n", hipGetErrorString(e));
        return -1;
    }
    return 0;
}

// The f32 chain (ftype 0 files, f32.hip): bert.cpp:963-1095 with every tensor in
// f32, the reference's own op order (QKV + bias, attention, (bias + O) + x, LN,
// GELU(bias + FFN-up), z + (bias + FFN-down), LN; mean pool, divide by the norm).
int Device::launch_all_f32(const int32_t *d_ids, const int32_t *d_cu, int n_seqs, int max_len, int T, float *d_out,
                           hipStream_t s)
{
    const int d = hp_.n_embd, f = hp_.n_intermediate;
    const int M = gemm_rows(T);
    const double t = (double)T;
    hipEvent_t ev;
    begin(K_EMBED_LN, s, ev);
    launch_f32_embed_ln(word_, type_, pos_, ln_e_w_, ln_e_b_, d_ids, d_cu, n_seqs, max_len, d, x32_, s);
    end(K_EMBED_LN, s, ev, t * (4.0 + 3.0 * d * 4.0 + 4.0 * d));
    for (int l = 0; l < hp_.n_layer; ++l) {
        const DevLayer &L = layers_[(size_t)l];
        begin(K_GEMM_QKV, s, ev);
        if (launch_f32_gemm(x32_, M, L.w32_qkv, 3 * d, d, L.b_qkv, 0, nullptr, qkv32_, s, gelu_tab_)) return -1;
        end(K_GEMM_QKV, s, ev, 2.0 * t * 3.0 * d * d);
        begin(K_ATTENTION, s, ev);
        if (launch_f32_attention(qkv32_, d_cu, n_seqs, max_len, hp_.n_head, d, att32_, s, exp_tab_)) return -1;
        end(K_ATTENTION, s, ev, att_flop_);
        begin(K_GEMM_O, s, ev);
        if (launch_f32_gemm(att32_, M, L.w32_o, d, d, L.b_o, 2, x32_, z32_, s, gelu_tab_)) return -1;
        end(K_GEMM_O, s, ev, 2.0 * t * d * d);
        begin(K_LN_STATS, s, ev);
        launch_f32_ln(z32_, M, d, L.ln1_w, L.ln1_b, s);
        end(K_LN_STATS, s, ev, (double)M * d * 8.0);
        begin(K_GEMM_FFN_UP, s, ev);
        if (launch_f32_gemm(z32_, M, L.w32_up, f, d, L.b_up, 1, nullptr, ffn32_, s, gelu_tab_)) return -1;
        end(K_GEMM_FFN_UP, s, ev, 2.0 * t * d * f);
        begin(K_GEMM_FFN_DOWN, s, ev);
        if (launch_f32_gemm(ffn32_, M, L.w32_down, d, f, L.b_down, 2, z32_, x32_, s, gelu_tab_)) return -1;
        end(K_GEMM_FFN_DOWN, s, ev, 2.0 * t * d * f);
        begin(K_LN_STATS, s, ev);
        launch_f32_ln(x32_, M, d, L.ln2_w, L.ln2_b, s);
        end(K_LN_STATS, s, ev, (double)M * d * 8.0);
    }
    begin(K_POOL_L2, s, ev);
    launch_f32_pool(x32_, d_cu, n_seqs, d, d_out, s);
    end(K_POOL_L2, s, ev, t * d * 4.0 + (double)n_seqs * d * 4.0);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        errorf("libbert: kernel launch failed: %s\n", hipGetErrorString(e));
        return -1;
    }
    return 0;
}

int Device::forward_host(const int32_t *const *tokens, const int32_t *lens, int n, float *const *out)
{
    if (!ok_) return -3;
    if (n <= 0) return 0;
    int64_t T = 0;
    int max_len = 0;
    double len2 = 0.0;
    for (int i = 0; i < n; ++i) {
        T += lens[i];
        max_len = std::max(max_len, (int)lens[i]);
        len2 += (double)lens[i] * lens[i];
    }
    DeviceGuard g(ordinal_);
    HIP_RC(g.status());
    if (!reserve(T, n, max_len)) return -1;
    order_after_last(stream_);   // the previous forward may have run on a caller stream
    h_cu_[0] = 0;
    for (int i = 0; i < n; ++i) {
        std::memcpy(h_ids_ + h_cu_[i], tokens[i], sizeof(int32_t) * (size_t)lens[i]);
        h_cu_[i + 1] = h_cu_[i] + lens[i];
    }
    HIP_RC(hipMemcpyAsync(d_ids_, h_ids_, sizeof(int32_t) * (size_t)T, hipMemcpyHostToDevice, stream_));
    HIP_RC(hipMemcpyAsync(d_cu_, h_cu_, sizeof(int32_t) * (size_t)(n + 1), hipMemcpyHostToDevice, stream_));
    const int rc = forward(d_ids_, d_cu_, n, max_len, (int)T, d_out_, stream_, len2);
    if (rc != 0) return rc;
    const size_t d = (size_t)hp_.n_embd;
    HIP_RC(hipMemcpyAsync(h_out_, d_out_, sizeof(float) * d * (size_t)n, hipMemcpyDeviceToHost, stream_));
    HIP_RC(hipStreamSynchronize(stream_));
    for (int i = 0; i < n; ++i) std::memcpy(out[i], h_out_ + d * (size_t)i, sizeof(float) * d);
    return 0;
}

}  // namespace emb

// ---------------------------------------------------------------------------
// per-kernel parity hooks (bert_hip.h): one GEMM on device 0, host buffers
// ---------------------------------------------------------------------------
#include "bert_hip.h"

namespace emb {
namespace {

// Device buffers of one hook call, freed together.
struct HookBufs {
    std::vector<void *> p;
    bool bad = false;
    void *up(const void *h, size_t bytes, size_t alloc)
    {
        void *d = nullptr;
        alloc = std::max<size_t>(std::max(alloc, bytes), 16);
        if (hipMalloc(&d, alloc) != hipSuccess) { bad = true; return nullptr; }
        p.push_back(d);
        if (hipMemset(d, 0, alloc) != hipSuccess) bad = true;
        if (h && bytes && hipMemcpy(d, h, bytes, hipMemcpyHostToDevice) != hipSuccess) bad = true;
        return d;
    }
    ~HookBufs() { for (void *d : p) (void)hipFree(d); }
};

// The weight of a hook call in the device layout; t keeps the file-format rows.
bool hook_weight(int32_t fmt, int32_t N, int32_t K, const void *w_rows, HostTensor &t, DevWeight &W, HookBufs &B)
{
    t.fmt = fmt; t.ne0 = K; t.ne1 = N;
    t.bytes.assign((const uint8_t *)w_rows, (const uint8_t *)w_rows + fmt_row_bytes(fmt, K) * (size_t)N);
    Piece q, dd, mm;
    repack_linear({&t}, fmt, q, dd, mm, W.N, W.K);
    W.fmt = fmt == FMT_F32 ? FMT_F16 : fmt;
    W.kx = fmt == FMT_F32 ? W.K / 2 : 0;
    W.qs = B.up(q.bytes.data(), q.bytes.size(), 0);
    W.d = (const uint16_t *)(dd.bytes.empty() ? nullptr : B.up(dd.bytes.data(), dd.bytes.size(), 0));
    W.m = (const uint16_t *)(mm.bytes.empty() ? nullptr : B.up(mm.bytes.data(), mm.bytes.size(), 0));
    return !B.bad;
}

HostTensor vec_tensor(const float *v, int n)
{
    HostTensor t;
    t.fmt = FMT_F32; t.ne0 = n; t.ne1 = 1;
    t.bytes.assign((const uint8_t *)v, (const uint8_t *)(v + n));
    return t;
}

}  // namespace
}  // namespace emb

extern "C" int32_t bertx_test_gemm(int32_t fmt, int32_t N, int32_t K, const void *w_rows, const float *bias,
                                   int32_t M, const uint16_t *x, int32_t epi, const void *res, void *out,
                                   int32_t cfg)
{
    return bertx_test_gemm_ln(fmt, N, K, w_rows, bias, M, x, nullptr, nullptr, nullptr, epi, (const uint16_t *)res,
                              nullptr, nullptr, nullptr, nullptr, (uint16_t *)out, nullptr, cfg);
}

extern "C" int32_t bertx_test_gemm_fold(int32_t fmt, int32_t N, int32_t K, const void *w_rows, const float *bias,
                                        int32_t M, const uint16_t *x, const float *part, const float *in_g,
                                        const float *in_b, int32_t epi, uint16_t *out, float *st_out,
                                        float *st_kernel, int32_t cfg)
{
    using namespace emb;
    if (!fmt_valid(fmt) || K % 64 || N % 32 || M <= 0 || (epi != 0 && epi != 1) || !part || !in_g || !in_b ||
        hip_device_count() == 0)
        return -1;
    const int Mp = (int)align_up((size_t)M, GEMM_BM), G = K / 32;   // (X columns: K for every format)
    DeviceGuard guard(0);
    HIP_RC(guard.status());
    HookBufs B;
    HostTensor t;
    DevWeight W;
    if (!hook_weight(fmt, N, K, w_rows, t, W, B)) return -1;
    g_gemm_cfg = cfg;
    const bool ok = gemm_fold_ok(W, Mp, G);
    g_gemm_cfg = 0;
    if (!ok) return -2;
    const HostTensor hb = vec_tensor(bias, N), hg = vec_tensor(in_g, K), hbt = vec_tensor(in_b, K);
    Piece c1, c2;
    fold_ln({&t}, {&hb}, hg, hbt, c1, c2, fmt == FMT_F32);
    LnFold ln;
    // partials [G][M] on the host -> [G][Mp] on the device (stride Mp)
    std::vector<float> hp((size_t)G * Mp * 2, 0.f);
    for (int g = 0; g < G; ++g) std::memcpy(&hp[(size_t)g * Mp * 2], part + (size_t)g * M * 2, (size_t)M * 8);
    ln.in_part = (const float2 *)B.up(hp.data(), hp.size() * 4, 0);
    ln.in_part_stride = Mp;
    ln.in_G = G;
    ln.st_out = (float2 *)B.up(nullptr, 0, (size_t)Mp * 8);
    ln.c1 = (const float *)B.up(c1.bytes.data(), c1.bytes.size(), 0);
    const float *dbias = (const float *)B.up(c2.bytes.data(), c2.bytes.size(), 0);
    void *dx = B.up(x, (size_t)M * K * 2, (size_t)Mp * K * 2);
    void *dout = B.up(nullptr, 0, (size_t)Mp * N * 2);
    if (B.bad) return -1;
    g_gemm_cfg = cfg;
    const int rc = launch_gemm(W, (const uint16_t *)dx, Mp, dbias, epi, nullptr, dout, nullptr, ln);
    g_gemm_cfg = 0;
    if (rc != 0) return rc;
    HIP_RC(hipGetLastError());
    HIP_RC(hipDeviceSynchronize());
    HIP_RC(hipMemcpy(out, dout, (size_t)M * N * 2, hipMemcpyDeviceToHost));
    if (st_out) HIP_RC(hipMemcpy(st_out, ln.st_out, (size_t)M * 8, hipMemcpyDeviceToHost));
    if (st_kernel) {
        // the same partials through the statistics kernel (the launch form)
        float2 *dk = (float2 *)B.up(nullptr, 0, (size_t)Mp * 8);
        if (B.bad || launch_ln_stats(ln.in_part, G, Mp, Mp, 32 * G, dk, nullptr) != 0) return -1;
        HIP_RC(hipDeviceSynchronize());
        HIP_RC(hipMemcpy(st_kernel, dk, (size_t)M * 8, hipMemcpyDeviceToHost));
    }
    return 0;
}

extern "C" int32_t bertx_test_gemm_ln(int32_t fmt, int32_t N, int32_t K, const void *w_rows, const float *bias,
                                      int32_t M, const uint16_t *x, const float *in_stats, const float *in_g,
                                      const float *in_b, int32_t epi, const uint16_t *res, const float *res_stats,
                                      const float *res_g, const float *res_b, const float *g_next, uint16_t *out,
                                      float *st_out, int32_t cfg)
{
    using namespace emb;
    if (!fmt_valid(fmt) || K % 64 || N % 32 || M <= 0 || epi < 0 || epi > 2 || hip_device_count() == 0) return -1;
    if (g_next && N > 1024) return -1;   // the statistics kernel combines at most 32 partials per row
    if ((in_stats && (!in_g || !in_b || epi == EPI_BIAS_RES)) || (epi == EPI_BIAS_RES && !res) ||
        (res_stats && (!res_g || !res_b)) || (g_next && epi != EPI_BIAS_RES))
        return -1;
    const int Mp = (int)align_up((size_t)M, GEMM_BM);
    DeviceGuard guard(0);
    HIP_RC(guard.status());
    HookBufs B;
    HostTensor t;
    DevWeight W;
    if (!hook_weight(fmt, N, K, w_rows, t, W, B)) return -1;
    LnFold ln;
    const float *dbias = (const float *)B.up(bias, (size_t)N * 4, 0);
    if (in_stats) {
        // the LN fold of the input: c1 = W gamma, c2 = bias + W beta
        const HostTensor hb = vec_tensor(bias, N), hg = vec_tensor(in_g, K), hbt = vec_tensor(in_b, K);
        Piece c1, c2;
        fold_ln({&t}, {&hb}, hg, hbt, c1, c2, fmt == FMT_F32);
        ln.in_stats = (const float2 *)B.up(in_stats, (size_t)M * 8, (size_t)Mp * 8);
        ln.c1 = (const float *)B.up(c1.bytes.data(), c1.bytes.size(), 0);
        dbias = (const float *)B.up(c2.bytes.data(), c2.bytes.size(), 0);
    }
    void *dx = B.up(x, (size_t)M * K * 2, (size_t)Mp * K * 2);
    void *dout = B.up(nullptr, 0, (size_t)Mp * N * 2);
    float2 *dst = nullptr;
    if (epi == EPI_BIAS_RES) {
        B.up(nullptr, 0, 0);
        void *dr = B.up(res, (size_t)M * N * 2, (size_t)Mp * N * 2);
        dout = dr;   // in place, as the forward runs it
        if (res_stats) {
            ln.res_stats = (const float2 *)B.up(res_stats, (size_t)M * 8, (size_t)Mp * 8);
            ln.res_g = (const float *)B.up(res_g, (size_t)N * 4, 0);
            ln.res_b = (const float *)B.up(res_b, (size_t)N * 4, 0);
        }
        if (g_next) {
            ln.g_next = (const float *)B.up(g_next, (size_t)N * 4, 0);
            ln.part = (float2 *)B.up(nullptr, 0, (size_t)Mp * (N / 32) * 8);
            ln.part_stride = Mp;
            dst = (float2 *)B.up(nullptr, 0, (size_t)Mp * 8);
        }
    }
    if (B.bad) return -1;
    g_gemm_cfg = cfg;
    const int rc = launch_gemm(W, (const uint16_t *)dx, Mp, dbias, epi, dout, dout, nullptr, ln);
    g_gemm_cfg = 0;
    if (rc != 0) return rc;
    if (dst && launch_ln_stats(ln.part, N / 32, Mp, Mp, N, dst, nullptr) != 0) return -1;
    HIP_RC(hipGetLastError());
    HIP_RC(hipDeviceSynchronize());
    HIP_RC(hipMemcpy(out, dout, (size_t)M * N * 2, hipMemcpyDeviceToHost));
    if (dst && st_out) HIP_RC(hipMemcpy(st_out, dst, (size_t)M * 8, hipMemcpyDeviceToHost));
    return 0;
}

extern "C" int32_t bertx_test_gemm_ran(void) { return emb::g_gemm_ran; }

// f32 chain GEMM (f32.hip) on host buffers: w f32 [N][K], x f32 [M][K], res/out f32 [M][N]
extern "C" int32_t bertx_test_gemm_f32(int32_t N, int32_t K, const float *w, const float *bias, int32_t M,
                                       const float *x, int32_t epi, const float *res, float *out)
{
    using namespace emb;
    if (N <= 0 || K % 32 || K <= 0 || M <= 0 || epi < 0 || epi > 2 || (epi == 2 && !res) || hip_device_count() == 0)
        return -1;
    const int Mp = (int)align_up((size_t)M, 64);
    DeviceGuard guard(0);
    HIP_RC(guard.status());
    HookBufs B;
    const float *dw = (const float *)B.up(w, (size_t)N * K * 4, 0);
    const float *db = (const float *)B.up(bias, (size_t)N * 4, 0);
    const float *dx = (const float *)B.up(x, (size_t)M * K * 4, (size_t)Mp * K * 4);
    const float *dr = epi == 2 ? (const float *)B.up(res, (size_t)M * N * 4, (size_t)Mp * N * 4) : nullptr;
    float *dout = (float *)B.up(nullptr, 0, (size_t)Mp * N * 4);
    std::vector<uint16_t> tg, te;
    era_tables(tg, te);
    const uint16_t *dg = (const uint16_t *)B.up(tg.data(), tg.size() * 2, 0);
    if (B.bad) return -1;
    if (launch_f32_gemm(dx, Mp, dw, N, K, db, epi, dr, dout, nullptr, dg) != 0) return -1;
    HIP_RC(hipGetLastError());
    HIP_RC(hipDeviceSynchronize());
    HIP_RC(hipMemcpy(out, dout, (size_t)M * N * 4, hipMemcpyDeviceToHost));
    return 0;
}

// ---------------------------------------------------------------------------
// GEMM micro-benchmark (bert_hip.h): device-timed launches on random operands,
// in the forward's own forms (LN fold on the input of epi 0/1; residual with
// its LN, the next gamma and the partial statistics for epi 2)
// ---------------------------------------------------------------------------
extern "C" int32_t bertx_bench_gemm(int32_t fmt, int32_t N, int32_t K, int32_t M, int32_t epi, int32_t cfg,
                                    int32_t iters, float *avg_us)
{
    using namespace emb;
    if (!fmt_valid(fmt) || K % 64 || N % 32 || M <= 0 || iters <= 0 || epi < 0 || epi > 2 ||
        hip_device_count() == 0)
        return -1;
    const int Mp = (int)align_up((size_t)M, GEMM_BM);
    uint32_t st = 12345u;
    auto rnd = [&]() { st = st * 1664525u + 1013904223u; return (st >> 8) / 16777216.0f; };
    // random weights in the file format, quantized by the native quantizer's rows
    std::vector<float> wrow((size_t)K);
    std::vector<uint8_t> rows(fmt_row_bytes(fmt, K) * (size_t)N);
    for (int n = 0; n < N; ++n) {
        for (auto &v : wrow) v = (rnd() - 0.5f) * 0.1f;
        quantize_row(fmt, wrow.data(), rows.data() + fmt_row_bytes(fmt, K) * (size_t)n, K);
    }
    std::vector<uint16_t> hx((size_t)Mp * K);
    for (auto &v : hx) v = f32_to_f16(rnd() - 0.5f);
    std::vector<float> hb((size_t)N), hg((size_t)std::max(N, K)), hbt((size_t)std::max(N, K)), hs((size_t)Mp * 2);
    for (auto &v : hb) v = (rnd() - 0.5f) * 0.1f;
    for (auto &v : hg) v = 1.0f + (rnd() - 0.5f) * 0.2f;
    for (auto &v : hbt) v = (rnd() - 0.5f) * 0.1f;
    for (size_t i = 0; i < hs.size(); i += 2) { hs[i] = 0.01f; hs[i + 1] = 1.0f + rnd() * 0.1f; }
    DeviceGuard guard(0);
    HIP_RC(guard.status());
    HookBufs B;
    HostTensor t;
    DevWeight W;
    if (!hook_weight(fmt, N, K, rows.data(), t, W, B)) return -1;
    LnFold ln;
    const float *dbias = (const float *)B.up(hb.data(), hb.size() * 4, 0);
    void *dx = B.up(hx.data(), hx.size() * 2, 0);
    void *dout = B.up(nullptr, 0, (size_t)Mp * N * 2);
    const bool plain = cfg & 0x100;   // A/B: the same GEMM without the LN fold
    cfg &= 0xff;
    if (plain) {
    } else if (epi == EPI_BIAS_RES) {
        ln.res_stats = (const float2 *)B.up(hs.data(), hs.size() * 4, 0);
        ln.res_g = (const float *)B.up(hg.data(), (size_t)N * 4, 0);
        ln.res_b = (const float *)B.up(hbt.data(), (size_t)N * 4, 0);
        ln.g_next = ln.res_g;
        ln.part = (float2 *)B.up(nullptr, 0, (size_t)Mp * (N / 32) * 8);
        ln.part_stride = Mp;
    } else {
        ln.in_stats = (const float2 *)B.up(hs.data(), hs.size() * 4, 0);
        ln.c1 = (const float *)B.up(hg.data(), (size_t)N * 4, 0);
    }
    if (B.bad) return -1;
    int lrc = 0;
    auto launch = [&]() {
        g_gemm_cfg = cfg;
        lrc |= launch_gemm(W, (const uint16_t *)dx, Mp, dbias, epi, dout, dout, nullptr, ln);
        g_gemm_cfg = 0;
    };
    for (int i = 0; i < 3; ++i) launch();
    if (lrc != 0) return -1;
    hipEvent_t a, b;
    HIP_RC(hipEventCreate(&a));
    HIP_RC(hipEventCreate(&b));
    HIP_RC(hipEventRecord(a, nullptr));
    for (int i = 0; i < iters; ++i) launch();
    HIP_RC(hipEventRecord(b, nullptr));
    HIP_RC(hipEventSynchronize(b));
    float ms = 0.f;
    HIP_RC(hipEventElapsedTime(&ms, a, b));
    *avg_us = ms * 1000.0f / (float)iters;
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// ---------------------------------------------------------------------------
// attention micro-benchmark (bert_hip.h): n_seqs sentences of `len` tokens,
// random Q/K/V, device-timed launches of variant `variant`
// ---------------------------------------------------------------------------
extern "C" int32_t bertx_bench_attention(int32_t n_seqs, int32_t len, int32_t n_head, int32_t dh, int32_t variant,
                                         int32_t iters, float *avg_us)
{
    using namespace emb;
    if (n_seqs <= 0 || len <= 0 || iters <= 0 || hip_device_count() == 0) return -1;
    const int d = n_head * dh;
    const size_t T = (size_t)n_seqs * len, rows = T + 256;
    std::vector<uint16_t> hq(rows * 3 * d);
    uint32_t st = 777u;
    for (auto &v : hq) { st = st * 1664525u + 1013904223u; v = f32_to_f16(((st >> 8) / 16777216.0f - 0.5f) * 2.0f); }
    std::vector<int32_t> hcu((size_t)n_seqs + 1);
    for (int i = 0; i <= n_seqs; ++i) hcu[(size_t)i] = i * len;
    uint16_t *dq = nullptr, *dout = nullptr;
    int32_t *dcu = nullptr;
    DeviceGuard guard(0);
    HIP_RC(guard.status());
    HIP_RC(hipMalloc((void **)&dq, hq.size() * 2));
    HIP_RC(hipMemcpy(dq, hq.data(), hq.size() * 2, hipMemcpyHostToDevice));
    HIP_RC(hipMalloc((void **)&dcu, hcu.size() * 4));
    HIP_RC(hipMemcpy(dcu, hcu.data(), hcu.size() * 4, hipMemcpyHostToDevice));
    HIP_RC(hipMalloc((void **)&dout, rows * d * 2));
    g_att_variant = variant;
    for (int i = 0; i < 3; ++i) launch_attention(dq, dcu, n_seqs, len, n_head, d, dout, nullptr);
    hipEvent_t a, b;
    HIP_RC(hipEventCreate(&a));
    HIP_RC(hipEventCreate(&b));
    HIP_RC(hipEventRecord(a, nullptr));
    for (int i = 0; i < iters; ++i) launch_attention(dq, dcu, n_seqs, len, n_head, d, dout, nullptr);
    HIP_RC(hipEventRecord(b, nullptr));
    HIP_RC(hipEventSynchronize(b));
    g_att_variant = 0;
    float ms = 0.f;
    HIP_RC(hipEventElapsedTime(&ms, a, b));
    *avg_us = ms * 1000.f / (float)iters;
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    for (void *p : {(void *)dq, (void *)dcu, (void *)dout}) (void)hipFree(p);
    return 0;
}

extern "C" int32_t bertx_test_attention(const uint16_t *qkv, const int32_t *cu, int32_t n_seqs, int32_t n_head,
                                        int32_t d, int32_t variant, uint16_t *out)
{
    using namespace emb;
    if (n_seqs <= 0 || n_head <= 0 || d % n_head || hip_device_count() == 0) return -1;
    const int dh = d / n_head;
    if (dh != 64 && dh != 32) return -1;
    int max_len = 0;
    for (int i = 0; i < n_seqs; ++i) {
        if (cu[i + 1] < cu[i]) return -1;
        max_len = std::max(max_len, cu[i + 1] - cu[i]);
    }
    const size_t T = (size_t)cu[n_seqs];
    uint16_t *dq = nullptr, *dout = nullptr;
    int32_t *dcu = nullptr;
    DeviceGuard guard(0);
    HIP_RC(guard.status());
    HIP_RC(hipMalloc((void **)&dq, (T + 64) * 3 * d * 2));
    HIP_RC(hipMemset(dq, 0, (T + 64) * 3 * d * 2));
    HIP_RC(hipMemcpy(dq, qkv, T * 3 * d * 2, hipMemcpyHostToDevice));
    HIP_RC(hipMalloc((void **)&dcu, ((size_t)n_seqs + 1) * 4));
    HIP_RC(hipMemcpy(dcu, cu, ((size_t)n_seqs + 1) * 4, hipMemcpyHostToDevice));
    HIP_RC(hipMalloc((void **)&dout, (T + 64) * d * 2));
    g_att_variant = variant;
    // variant -1: the streaming kernel, reached by claiming a length past the LDS form
    launch_attention(dq, dcu, n_seqs, variant == -1 ? ATT_LDS_MAX + 1 : max_len, n_head, d, dout, nullptr);
    g_att_variant = 0;
    HIP_RC(hipDeviceSynchronize());
    HIP_RC(hipMemcpy(out, dout, T * d * 2, hipMemcpyDeviceToHost));
    for (void *p : {(void *)dq, (void *)dcu, (void *)dout}) (void)hipFree(p);
    return 0;
}
