/* ASan/UBSan harness of the C oracle (test infrastructure, oracle/bert_oracle.c):
 *   fwd <model.bin> <ids.bin> <out.bin>   ids: u32 n, (u32 len, i32 ids[len])*n;
 *                                         out: n x n_embd f32 (bert_forward_batch)
 * Built by tests/sanitize/Makefile, driven by tests/test_cpu_sanitize.py. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct omodel omodel;
omodel *oracle_load(const char *path);
void oracle_free(omodel *m);
void oracle_hparams(omodel *m, int32_t *out7);
int oracle_forward_batch(omodel *m, int n_threads, int n, const int32_t *flat, const int32_t *lens, float *out);

int main(int argc, char **argv)
{
    if (argc != 5 || strcmp(argv[1], "fwd") != 0) return 1;
    omodel *m = oracle_load(argv[2]);
    if (!m) return 2;
    int32_t hp[7];
    oracle_hparams(m, hp);
    FILE *f = fopen(argv[3], "rb");
    uint32_t n = 0;
    if (!f || fread(&n, 4, 1, f) != 1) return 3;
    int32_t *lens = calloc(n, sizeof(int32_t));
    size_t tot = 0, cap = 1024;
    int32_t *flat = malloc(cap * sizeof(int32_t));
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t len = 0;
        if (fread(&len, 4, 1, f) != 1) return 3;
        while (tot + len > cap) { cap *= 2; flat = realloc(flat, cap * sizeof(int32_t)); }
        if (len && fread(flat + tot, 4, len, f) != len) return 3;
        lens[i] = (int32_t)len;
        tot += len;
    }
    fclose(f);
    float *out = calloc((size_t)n * hp[2], sizeof(float));
    const int rc = oracle_forward_batch(m, 2, (int)n, flat, lens, out);
    FILE *o = fopen(argv[4], "wb");
    if (!o) return 4;
    fwrite(out, sizeof(float), (size_t)n * hp[2], o);
    fclose(o);
    free(out);
    free(flat);
    free(lens);
    oracle_free(m);
    return rc;
}
