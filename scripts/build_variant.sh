#!/usr/bin/env bash
# A/B build of libbert.so with extra defines: build_ab/NAME/libbert.so
# usage: scripts/build_variant.sh NAME "-DFOO=1 -DBAR=2"; run with BERT_LIB=build_ab/NAME/libbert.so
set -euo pipefail
cd "$(dirname "$0")/.."
make -s -j8 -C embeddings.cpp_amd BUILD="$(pwd)/build_ab/$1" EXTRA="$2" "$(pwd)/build_ab/$1/libbert.so"
