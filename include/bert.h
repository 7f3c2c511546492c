/*
 * bert.h — drop-in C ABI of the MI355X-native embedding engine (libbert.so).
 *
 * Every declaration below keeps the exact name, argument order, types and
 * calling convention of snowyu/embeddings.cpp's bert.h (reference bert.h:18-90),
 * so the reference's callers link or dlopen this library unchanged:
 *   - examples/sample_dylib.py / benchmarks/run_mteb.py (ctypes, 4 symbols),
 *   - examples/dylib.cpp (dlsym), examples/server.cpp, main.cpp, test_*.cpp.
 *
 * Semantics follow the reference; GPU-specific notes are marked [MI355X].
 */
#ifndef BERT_H
#define BERT_H

#include <stddef.h>
#include <stdint.h>
#include <stdbool.h>

#if defined(_WIN32)
#define BERT_API __declspec(dllexport)
#else
#define BERT_API __attribute__((visibility("default")))
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* CLI parameters (reference bert.h:18-25; defaults identical).  The default
 * member initialisers make this header C++-only, exactly like the reference. */
struct bert_params
{
    int32_t n_threads = 6;
    int32_t port = 8080;
    const char *model = "models/all-MiniLM-L6-v2/ggml-model-q4_0.bin";
    const char *prompt = "test prompt";
};

/* -t/--threads, -p/--prompt, --port, -m/--model, -h/--help; an unknown flag
 * prints usage and exits(0) (reference bert.cpp:157-193). */
BERT_API bool bert_params_parse(int argc, char **argv, bert_params &params);

/* Opaque context.  [MI355X] holds the vocab on the host and a weight replica +
 * workspace + HIP stream per GPU selected by BERT_DEVICES (default: all). */
struct bert_ctx;

typedef int32_t bert_vocab_id;

/* Parses a ggml-era model file (magic 0x67676d6c, reference bert.cpp:423-786):
 * ftype 0 f32, 1 f16, 2 q4_0, 3 q4_1, and 8 q8_0 (extension).  Returns NULL
 * on any error.  [MI355X] fails loudly (NULL) when no HIP device is present,
 * unless BERT_HOST_ONLY=1 (tokenizer-only context; every forward then prints
 * an error and leaves its outputs unwritten). */
BERT_API struct bert_ctx *bert_load_from_file(const char *fname);
BERT_API void bert_free(bert_ctx *ctx);

/* One text -> one float[n_embd] (reference bert.cpp:1365-1372). */
BERT_API void bert_encode(
    struct bert_ctx *ctx,
    int32_t n_threads,
    const char *texts,
    float *embeddings);

/* n_inputs texts -> embeddings[i] = float[n_embd] (reference bert.cpp:1374-1444).
 * Chunks of n_batch_size in ascending token length unless
 * n_batch_size == n_inputs; a chunk holding an input longer than
 * n_max_tokens is refused (outputs left untouched), as in the reference.
 * [MI355X] n_threads sizes the host tokenizer pool; sentences are sharded over
 * the context's GPUs by cost. */
BERT_API void bert_encode_batch(
    struct bert_ctx *ctx,
    int32_t n_threads,
    int32_t n_batch_size,
    int32_t n_inputs,
    const char **texts,
    float **embeddings);

/* WordPiece tokenizer, bit-exact to reference bert.cpp:297-417 ([CLS]=101,
 * [SEP]=102, [UNK]=100).  *n_tokens gets the reference's full count (it can
 * exceed n_max_tokens for long multi-word inputs, bert.cpp:386-412);
 * [MI355X] at most n_max_tokens ids are stored into `tokens`. */
BERT_API void bert_tokenize(
    struct bert_ctx *ctx,
    const char *text,
    bert_vocab_id *tokens,
    int32_t *n_tokens,
    int32_t n_max_tokens);

/* Single-sequence forward (reference bert.cpp:817-825).  embeddings may be
 * NULL (the reference's memory-measurement mode): nothing is written. */
BERT_API void bert_forward(
    struct bert_ctx *ctx,
    int32_t n_threads,
    bert_vocab_id *tokens,
    int32_t n_tokens,
    float *embeddings);

/* Batched forward of pre-tokenized inputs (reference bert.cpp:827-1147):
 * token+type(0)+position embeddings, LayerNorm, n_layer encoder layers,
 * masked mean pool, L2 normalise.  Refused (no output) when the longest input
 * exceeds n_max_tokens.  [MI355X] inputs need not be sorted. */
BERT_API void bert_forward_batch(
    struct bert_ctx *ctx,
    int32_t n_threads,
    int32_t n_batch_size,
    bert_vocab_id **batch_tokens,
    int32_t *n_tokens,
    float **batch_embeddings);

/* Reference bert.cpp:1151-1363: same math, one unmasked graph per input.
 * [MI355X] runs the same GPU kernels (per-sentence masking is exact). */
BERT_API void bert_forward_fake_batch(
    struct bert_ctx *ctx,
    int32_t n_threads,
    int32_t n_batch_size,
    bert_vocab_id **batch_tokens,
    int32_t *n_tokens,
    float **batch_embeddings);

BERT_API int32_t bert_n_embd(bert_ctx *ctx);
BERT_API int32_t bert_n_max_tokens(bert_ctx *ctx);

/* Reference bert.cpp:121-134, including its "[UNK TOKEN from bert_vocab]". */
BERT_API const char *bert_vocab_id_to_token(bert_ctx *ctx, bert_vocab_id id);

#ifdef __cplusplus
}
#endif

#endif /* BERT_H */
