// build/bin/convert — the command line of models/convert-to-ggml.py:9-16,43-50:
//   convert dir-model [ftype]     ftype 0 = f32, 1 = f16 (default)
// writes dir-model/ggml-model-{f32,f16}.bin, or dir-model/ggml-model.bin when
// ftype is omitted (the script's fname_out before the argument is parsed).
// Reads only a local directory: there is no hub download.
#include "bert_hip.h"

#include <cstdio>
#include <cstdlib>
#include <string>

int main(int argc, char **argv)
{
    if (argc < 2) {
        std::printf("Usage: convert dir-model [use-f32]\n\n");
        std::printf("  ftype == 0 -> float32\n  ftype == 1 -> float16\n");
        return 1;
    }
    const std::string dir = argv[1];
    int ftype = 1;
    std::string out = dir + "/ggml-model.bin";
    if (argc > 2) {
        ftype = std::atoi(argv[2]);
        if (ftype < 0 || ftype > 1) {
            std::printf("Invalid ftype: %d\n", ftype);
            return 1;
        }
        out = dir + (ftype == 0 ? "/ggml-model-f32.bin" : "/ggml-model-f16.bin");
    }
    if (bertx_convert_hf(dir.c_str(), out.c_str(), ftype) != 0) return 1;
    std::printf("Done. Output file: %s\n\n", out.c_str());
    return 0;
}
