// Native HF -> model-file converter.  Restates what
// models/convert-to-ggml.py:1-113 writes, without Python/torch:
//   * header: magic, 7 int32 hparams from config.json (convert-to-ggml.py:68-75);
//   * vocab: hparams.vocab_size lines of vocab.txt, each with its last
//     character dropped (`vocab[i][:-1]`, :77-81 -- text-mode readlines, so
//     "\r\n" and a lone "\r" are line ends too);
//   * tensors in BertModel.state_dict() order, skipping position_ids and the
//     pooler (:85-87); size-1 dims squeezed (:84); 2-D "*.weight" stored f16
//     when ftype == 1, everything else f32 (:91-97); dims written fastest-first
//     (:100-102), then the name and the raw data.
// Input: model.safetensors (or a sharded model.safetensors.index.json) --
// pickled pytorch_model.bin checkpoints are not read (nothing that unpickles
// runs here).  F32/F16/BF16/F64 tensors are widened to f32 first, so a
// half-precision checkpoint converts as if it had been loaded in f32.
#include "host_common.h"

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

namespace emb {

namespace {

// ---- minimal JSON (objects, arrays, strings, numbers, literals) ----
struct JVal {
    enum Kind { NUL, BOOL, NUM, STR, ARR, OBJ } kind = NUL;
    double num = 0;
    bool b = false;
    std::string str;
    std::vector<JVal> arr;
    std::vector<std::pair<std::string, JVal>> obj;   // keeps file order
    const JVal *get(const std::string &k) const
    {
        for (auto &kv : obj)
            if (kv.first == k) return &kv.second;
        return nullptr;
    }
};

struct JParser {
    const char *p, *e;
    bool ok = true;
    void ws() { while (p < e && std::isspace((unsigned char)*p)) ++p; }
    bool lit(const char *s)
    {
        const size_t n = std::strlen(s);
        if ((size_t)(e - p) < n || std::memcmp(p, s, n) != 0) return false;
        p += n;
        return true;
    }
    static void put_utf8(std::string &o, uint32_t c)
    {
        if (c < 0x80) o += (char)c;
        else if (c < 0x800) { o += (char)(0xc0 | (c >> 6)); o += (char)(0x80 | (c & 63)); }
        else if (c < 0x10000) {
            o += (char)(0xe0 | (c >> 12)); o += (char)(0x80 | ((c >> 6) & 63)); o += (char)(0x80 | (c & 63));
        } else {
            o += (char)(0xf0 | (c >> 18)); o += (char)(0x80 | ((c >> 12) & 63));
            o += (char)(0x80 | ((c >> 6) & 63)); o += (char)(0x80 | (c & 63));
        }
    }
    uint32_t hex4()
    {
        if (e - p < 4) { ok = false; return 0; }
        uint32_t v = 0;
        for (int i = 0; i < 4; ++i) {
            const char c = *p++;
            v <<= 4;
            if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
            else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
            else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
            else ok = false;
        }
        return v;
    }
    std::string string()
    {
        std::string o;
        ++p;   // opening quote
        while (p < e && *p != '"') {
            if (*p != '\\') { o += *p++; continue; }
            if (++p >= e) break;
            const char c = *p++;
            switch (c) {
            case 'n': o += '\n'; break;
            case 't': o += '\t'; break;
            case 'r': o += '\r'; break;
            case 'b': o += '\b'; break;
            case 'f': o += '\f'; break;
            case 'u': {
                uint32_t u = hex4();
                if (u >= 0xd800 && u < 0xdc00 && e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
                    p += 2;
                    const uint32_t lo = hex4();
                    u = 0x10000 + ((u - 0xd800) << 10) + (lo - 0xdc00);
                }
                put_utf8(o, u);
                break;
            }
            default: o += c;
            }
        }
        if (p >= e) ok = false;
        else ++p;
        return o;
    }
    JVal value(int depth = 0)
    {
        JVal v;
        ws();
        if (p >= e || depth > 64) { ok = false; return v; }
        if (*p == '{') {
            v.kind = JVal::OBJ;
            ++p;
            ws();
            if (p < e && *p == '}') { ++p; return v; }
            while (ok) {
                ws();
                if (p >= e || *p != '"') { ok = false; break; }
                std::string k = string();
                ws();
                if (p >= e || *p != ':') { ok = false; break; }
                ++p;
                v.obj.emplace_back(std::move(k), value(depth + 1));
                ws();
                if (p < e && *p == ',') { ++p; continue; }
                if (p < e && *p == '}') { ++p; break; }
                ok = false;
            }
        } else if (*p == '[') {
            v.kind = JVal::ARR;
            ++p;
            ws();
            if (p < e && *p == ']') { ++p; return v; }
            while (ok) {
                v.arr.push_back(value(depth + 1));
                ws();
                if (p < e && *p == ',') { ++p; continue; }
                if (p < e && *p == ']') { ++p; break; }
                ok = false;
            }
        } else if (*p == '"') {
            v.kind = JVal::STR;
            v.str = string();
        } else if (lit("true")) { v.kind = JVal::BOOL; v.b = true; }
        else if (lit("false")) { v.kind = JVal::BOOL; }
        else if (lit("null")) { v.kind = JVal::NUL; }
        else {
            char *end = nullptr;
            const std::string tmp(p, (size_t)std::min<ptrdiff_t>(e - p, 64));
            v.num = std::strtod(tmp.c_str(), &end);
            if (end == tmp.c_str()) { ok = false; return v; }
            v.kind = JVal::NUM;
            p += end - tmp.c_str();
        }
        return v;
    }
};

bool parse_json(const std::string &s, JVal &out)
{
    JParser jp{s.data(), s.data() + s.size()};
    out = jp.value();
    return jp.ok && out.kind == JVal::OBJ;
}

bool read_file(const std::string &path, std::string &out)
{
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::ostringstream ss;
    ss << f.rdbuf();
    out = ss.str();
    return true;
}

float bf16_to_f32(uint16_t h)
{
    const uint32_t x = (uint32_t)h << 16;
    float f;
    std::memcpy(&f, &x, 4);
    return f;
}

struct StTensor {
    std::vector<int64_t> shape;
    std::vector<float> data;   // widened to f32
};

// one safetensors file: u64 header length, JSON header, raw little-endian data
bool load_safetensors(const std::string &path, std::map<std::string, StTensor> &out)
{
    std::string raw;
    if (!read_file(path, raw) || raw.size() < 8) {
        errorf("convert: cannot read '%s'\n", path.c_str());
        return false;
    }
    uint64_t hlen;
    std::memcpy(&hlen, raw.data(), 8);
    if (hlen > raw.size() - 8) return false;
    JVal hdr;
    if (!parse_json(raw.substr(8, hlen), hdr)) {
        errorf("convert: bad safetensors header in '%s'\n", path.c_str());
        return false;
    }
    const char *base = raw.data() + 8 + hlen;
    const size_t avail = raw.size() - 8 - hlen;
    for (auto &kv : hdr.obj) {
        if (kv.first == "__metadata__") continue;
        const JVal *dt = kv.second.get("dtype"), *sh = kv.second.get("shape"), *off = kv.second.get("data_offsets");
        if (!dt || !sh || !off || off->arr.size() != 2) return false;
        StTensor t;
        int64_t n = 1;
        for (auto &d : sh->arr) { t.shape.push_back((int64_t)d.num); n *= (int64_t)d.num; }
        const size_t a = (size_t)off->arr[0].num, b = (size_t)off->arr[1].num;
        if (b < a || b > avail) return false;
        const char *src = base + a;
        t.data.resize((size_t)n);
        size_t esz;
        if (dt->str == "F32") esz = 4;
        else if (dt->str == "F16" || dt->str == "BF16") esz = 2;
        else if (dt->str == "F64") esz = 8;
        else {
            errorf("convert: tensor '%s' has unsupported dtype %s\n", kv.first.c_str(),
                         dt->str.c_str());
            return false;
        }
        if ((size_t)n * esz != b - a) return false;
        for (int64_t i = 0; i < n; ++i) {
            const char *q = src + (size_t)i * esz;
            if (esz == 4) std::memcpy(&t.data[(size_t)i], q, 4);
            else if (esz == 8) { double d; std::memcpy(&d, q, 8); t.data[(size_t)i] = (float)d; }
            else {
                uint16_t h;
                std::memcpy(&h, q, 2);
                t.data[(size_t)i] = dt->str == "F16" ? f16_to_f32(h) : bf16_to_f32(h);
            }
        }
        out[kv.first] = std::move(t);
    }
    return true;
}

// checkpoint names -> BertModel state_dict names (what AutoModel would load):
// a task-head prefix "bert." is dropped, legacy LayerNorm gamma/beta renamed.
std::string canonical_name(std::string n)
{
    if (n.rfind("bert.", 0) == 0) n = n.substr(5);
    auto ends = [&](const char *s) {
        const size_t k = std::strlen(s);
        return n.size() >= k && n.compare(n.size() - k, k, s) == 0;
    };
    if (ends("LayerNorm.gamma")) n = n.substr(0, n.size() - 5) + "weight";
    else if (ends("LayerNorm.beta")) n = n.substr(0, n.size() - 4) + "bias";
    return n;
}

// BertModel registration order (modeling_bert BertEmbeddings / BertLayer)
std::vector<std::string> state_dict_order(int n_layer)
{
    std::vector<std::string> v = {"embeddings.word_embeddings.weight", "embeddings.position_embeddings.weight",
                                  "embeddings.token_type_embeddings.weight", "embeddings.LayerNorm.weight",
                                  "embeddings.LayerNorm.bias"};
    const char *sub[] = {"attention.self.query", "attention.self.key", "attention.self.value",
                         "attention.output.dense", "attention.output.LayerNorm", "intermediate.dense",
                         "output.dense", "output.LayerNorm"};
    for (int l = 0; l < n_layer; ++l)
        for (const char *s : sub)
            for (const char *wb : {".weight", ".bias"})
                v.push_back("encoder.layer." + std::to_string(l) + "." + s + wb);
    return v;
}

template <typename T> void put(std::string &o, const T &v) { o.append((const char *)&v, sizeof(T)); }

}  // namespace

int convert_hf_dir(const std::string &dir, const std::string &fname_out, int ftype)
{
    if (ftype < 0 || ftype > 1) {
        errorf("Invalid ftype: %d\n", ftype);
        return 1;
    }
    std::string s;
    JVal cfg;
    if (!read_file(dir + "/config.json", s) || !parse_json(s, cfg)) {
        errorf("convert: cannot read %s/config.json\n", dir.c_str());
        return 1;
    }
    const char *keys[] = {"vocab_size", "max_position_embeddings", "hidden_size", "intermediate_size",
                          "num_attention_heads", "num_hidden_layers"};
    int32_t hp[6];
    for (int i = 0; i < 6; ++i) {
        const JVal *v = cfg.get(keys[i]);
        if (!v || v->kind != JVal::NUM) {
            errorf("convert: config.json lacks %s\n", keys[i]);
            return 1;
        }
        hp[i] = (int32_t)v->num;
    }

    // vocab.txt in text mode: universal newlines, each line keeps its "\n"
    if (!read_file(dir + "/vocab.txt", s)) {
        errorf("convert: cannot read %s/vocab.txt\n", dir.c_str());
        return 1;
    }
    std::vector<std::string> lines;
    {
        std::string cur;
        for (size_t i = 0; i < s.size(); ++i) {
            const char c = s[i];
            if (c == '\r' || c == '\n') {
                if (c == '\r' && i + 1 < s.size() && s[i + 1] == '\n') ++i;
                lines.push_back(cur + "\n");
                cur.clear();
            } else cur += c;
        }
        if (!cur.empty()) lines.push_back(cur);
    }
    if ((int64_t)lines.size() < hp[0]) {
        errorf("convert: vocab.txt has %zu lines, config says vocab_size %d\n", lines.size(), hp[0]);
        return 1;
    }

    // tensors: one file or a sharded index
    std::map<std::string, StTensor> raw;
    JVal idx;
    if (read_file(dir + "/model.safetensors.index.json", s)) {
        if (!parse_json(s, idx) || !idx.get("weight_map")) return 1;
        std::vector<std::string> shards;
        for (auto &kv : idx.get("weight_map")->obj)
            if (std::find(shards.begin(), shards.end(), kv.second.str) == shards.end())
                shards.push_back(kv.second.str);
        for (auto &f : shards)
            if (!load_safetensors(dir + "/" + f, raw)) return 1;
    } else if (!load_safetensors(dir + "/model.safetensors", raw)) {
        errorf("convert: %s has no model.safetensors (pickled checkpoints are not read)\n",
                     dir.c_str());
        return 1;
    }
    std::map<std::string, StTensor *> byname;
    for (auto &kv : raw) byname[canonical_name(kv.first)] = &kv.second;

    std::vector<std::string> order = state_dict_order(hp[5]);
    for (auto &n : order)
        if (!byname.count(n)) {
            errorf("convert: checkpoint lacks tensor '%s'\n", n.c_str());
            return 1;
        }
    // anything else BertModel would hold (not the pooler / position_ids / task heads)
    for (auto &kv : byname) {
        const std::string &n = kv.first;
        if (std::find(order.begin(), order.end(), n) != order.end()) continue;
        if (n == "embeddings.position_ids" || n.rfind("pooler.", 0) == 0 || n.rfind("cls.", 0) == 0) continue;
        if (n.rfind("embeddings.", 0) == 0 || n.rfind("encoder.", 0) == 0) order.push_back(n);
    }

    std::string o;
    put(o, (int32_t)0x67676d6c);
    for (int i = 0; i < 6; ++i) put(o, hp[i]);
    put(o, (int32_t)ftype);
    for (int i = 0; i < hp[0]; ++i) {
        const std::string &l = lines[(size_t)i];
        const std::string text = l.substr(0, l.size() - 1);
        put(o, (int32_t)text.size());
        o += text;
    }
    for (auto &n : order) {
        const StTensor &t = *byname[n];
        std::vector<int64_t> dims;            // squeeze()
        for (int64_t d : t.shape)
            if (d != 1) dims.push_back(d);
        const int nd = (int)dims.size();
        const bool half = ftype == 1 && nd == 2 && n.size() >= 7 && n.compare(n.size() - 7, 7, ".weight") == 0;
        put(o, (int32_t)nd);
        put(o, (int32_t)n.size());
        put(o, (int32_t)(half ? 1 : 0));
        for (int i = nd - 1; i >= 0; --i) put(o, (int32_t)dims[(size_t)i]);
        o += n;
        if (half)
            for (float v : t.data) put(o, f32_to_f16(v));
        else
            o.append((const char *)t.data.data(), t.data.size() * 4);
    }
    FILE *f = std::fopen(fname_out.c_str(), "wb");
    if (!f) {
        errorf("convert: cannot open '%s' for writing\n", fname_out.c_str());
        return 1;
    }
    const bool ok = std::fwrite(o.data(), 1, o.size(), f) == o.size();
    std::fclose(f);
    return ok ? 0 : 1;
}

}  // namespace emb
