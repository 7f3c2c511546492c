// build/bin/quantize — same command line as the reference's models/quantize.cpp
// (main at quantize.cpp:273-319):  quantize model-f32.bin model-quant.bin type
// type = 2 (q4_0), 3 (q4_1), 8 (q8_0, extension).
#include "bert_hip.h"

#include <cstdio>
#include <cstdlib>

int main(int argc, char **argv)
{
    if (argc != 4) {
        std::fprintf(stderr, "usage: %s model-f32.bin model-quant.bin type\n", argv[0]);
        std::fprintf(stderr, "  type = 2 - q4_0\n  type = 3 - q4_1\n  type = 8 - q8_0 (extension)\n");
        return 1;
    }
    const int rc = bertx_quantize_file(argv[1], argv[2], std::atoi(argv[3]));
    if (rc != 0) std::fprintf(stderr, "%s: failed to quantize model from '%s'\n", argv[0], argv[1]);
    return rc == 0 ? 0 : 1;
}
