#!/usr/bin/env bash
# Drop-in check: compile the reference's OWN example programs, unmodified, from
# /root/reference/examples against include/bert.h + include/ggml.h and link them
# to build/libbert.so -- what a maintainer does after swapping the library.
# Outputs only into build/ref_clients/ (git-ignored; travels to the GPU box with
# the snapshot).  Reference sources are read in place, never copied.
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
REF="${REF:-/root/reference}"
OUT="$ROOT/build/ref_clients"
[ -d "$REF/examples" ] || { echo "no reference checkout at $REF; skipping"; exit 0; }
[ -f "$ROOT/build/libbert.so" ] || make -C "$ROOT/embeddings.cpp_amd" -j8
mkdir -p "$OUT"
for p in server main test_batch_encode test_tokenizer; do
  g++ -O2 -std=c++17 -I"$ROOT/include" "$REF/examples/$p.cpp" -o "$OUT/$p" \
      -L"$ROOT/build" -lbert -Wl,-rpath,'$ORIGIN/..'
done
# dylib.cpp dlopen()s "../build/libbert.so" relative to its working directory
g++ -O2 -std=c++17 "$REF/examples/dylib.cpp" -o "$OUT/dylib" -ldl
echo "built $(ls "$OUT" | tr '\n' ' ')in $OUT"
