// ORACLE-SIDE HARNESS — TEST INFRASTRUCTURE ONLY.
//
// Compiles the reference's OWN tokenizer source (bert.cpp:195-417), its vocab
// insertion rule (bert.cpp:483-493) and bert_vocab_id_to_token (bert.cpp:121-134)
// straight from /root/reference.  oracle/build_ref.sh extracts those line ranges
// into a temporary directory at build time (they contain no ggml code) and
// compiles this file against them; only the resulting oracle/_ref/libreftok.so
// is kept (git-ignored).  No reference source is stored in this repository.
//
// `struct bert_ctx` here holds only the `vocab` member the tokenizer touches;
// the real struct (bert.cpp:100-109) also holds ggml model state, which the
// tokenizer never reads.
#include "bert.h"

#include <cctype>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "vocab_struct.inc"      // bert.cpp:57-64  (struct bert_vocab)

struct bert_ctx {
    bert_vocab vocab;
};

#include "id_to_token.inc"       // bert.cpp:121-134
#include "tokenizer.inc"         // bert.cpp:195-417

extern "C" {

__attribute__((visibility("default"))) bert_ctx *reftok_new() { return new bert_ctx; }
__attribute__((visibility("default"))) void reftok_free(bert_ctx *c) { delete c; }

// One vocab entry exactly as the loader inserts it (bert.cpp:475-494 loop body).
__attribute__((visibility("default"))) void reftok_add(bert_ctx *ctx, const char *data, uint32_t len, int i)
{
    bert_vocab &vocab = ctx->vocab;
    std::string word(data, len);
#include "vocab_insert.inc"      // bert.cpp:483-493
}

__attribute__((visibility("default"))) void reftok_tokenize(bert_ctx *ctx, const char *text, int32_t *tokens,
                                                            int32_t *n_tokens, int32_t n_max_tokens)
{
    bert_tokenize(ctx, text, tokens, n_tokens, n_max_tokens);
}

__attribute__((visibility("default"))) const char *reftok_id_to_token(bert_ctx *ctx, int32_t id)
{
    return bert_vocab_id_to_token(ctx, id);
}
}
