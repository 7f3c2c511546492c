// ASan/UBSan harness of libbert's host code (test infrastructure): the tokenizer
// (tokenizer.cpp), the model-file loader and quantizer (model_file.cpp) and the
// converter (converter.cpp), built with -fsanitize=address,undefined by
// tests/sanitize/Makefile and driven by tests/test_cpu_sanitize.py.
//   tok <vocab.bin> <texts.bin> <ids.bin>   vocab: u32 n, (u32 len, bytes)*n;
//                                          texts: u32 n, (i32 n_max, u32 len, bytes)*n;
//                                          ids: per text i32 count, then min(count, n_max) i32
//   load <model.bin>                       parse a model file, print hparams and tensor count
//   quant <in.bin> <out.bin> <itype>       the native quantizer
//   convert <hf_dir> <out.bin> <ftype>     the native converter
#include "host_common.h"
#include "tokenizer.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

using namespace emb;

static bool rd(FILE *f, void *p, size_t n) { return n == 0 || std::fread(p, 1, n, f) == n; }

static int cmd_tok(const char *vf, const char *tf, const char *of)
{
    FILE *v = std::fopen(vf, "rb"), *t = std::fopen(tf, "rb"), *o = std::fopen(of, "wb");
    if (!v || !t || !o) return 2;
    uint32_t n = 0, len = 0;
    std::vector<std::string> vocab;
    if (!rd(v, &n, 4)) return 3;
    for (uint32_t i = 0; i < n; ++i) {
        if (!rd(v, &len, 4)) return 3;
        std::string s(len, '\0');
        if (!rd(v, &s[0], len)) return 3;
        vocab.push_back(s);
    }
    Vocab voc;
    voc.build(vocab);
    for (uint32_t i = 0; i < n; ++i)
        if (!voc.id_to_token((int32_t)i)) return 4;
    if (!rd(t, &n, 4)) return 3;
    for (uint32_t i = 0; i < n; ++i) {
        int32_t nmax = 0;
        if (!rd(t, &nmax, 4) || !rd(t, &len, 4)) return 3;
        // an exact-size heap buffer, so a read past the terminator is a reported error
        std::vector<char> text(len + 1);
        if (!rd(t, text.data(), len)) return 3;
        text[len] = 0;
        std::vector<int32_t> ids((size_t)(nmax > 0 ? nmax : 0));
        const int32_t cnt = voc.tokenize(text.data(), nmax, ids.data(), nmax > 0 ? nmax : 0);
        std::fwrite(&cnt, 4, 1, o);
        const int32_t w = cnt < nmax ? cnt : nmax;
        if (w > 0) std::fwrite(ids.data(), 4, (size_t)w, o);
    }
    std::fclose(v);
    std::fclose(t);
    std::fclose(o);
    return 0;
}

int main(int argc, char **argv)
{
    if (argc < 3) return 1;
    const std::string c = argv[1];
    if (c == "tok" && argc == 5) return cmd_tok(argv[2], argv[3], argv[4]);
    if (c == "load") {
        HostModel m;
        std::string err;
        if (!load_model_file(argv[2], m, err, false)) {
            std::fprintf(stderr, "load failed: %s\n", err.c_str());
            return 5;
        }
        std::vector<float> row;
        for (const HostLayer &L : m.layers) {   // every weight row dequantizes
            row.resize((size_t)L.i_w.ne0);
            for (int r = 0; r < L.i_w.ne1; ++r)
                dequant_row(L.i_w.fmt, L.i_w.bytes.data() + fmt_row_bytes(L.i_w.fmt, L.i_w.ne0) * r, row.data(),
                            L.i_w.ne0);
        }
        std::printf("%d %d %d %d %d %d %d %d\n", m.hp.n_vocab, m.hp.n_max_tokens, m.hp.n_embd, m.hp.n_intermediate,
                    m.hp.n_head, m.hp.n_layer, m.hp.ftype, m.n_tensors);
        return 0;
    }
    if (c == "quant" && argc == 5) return quantize_file(argv[2], argv[3], std::atoi(argv[4]), false);
    if (c == "convert" && argc == 5) return convert_hf_dir(argv[2], argv[3], std::atoi(argv[4]));
    return 1;
}
