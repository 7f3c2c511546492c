#!/usr/bin/env bash
# Builds oracle/_ref/libreftok.so from the reference's own tokenizer source
# (ORACLE / test infrastructure only).  Needs /root/reference; the extracted
# source lines live only in a temp dir and are deleted afterwards.
set -euo pipefail
REF=${REF:-/root/reference}
HERE="$(cd "$(dirname "$0")" && pwd)"
OUT="$HERE/_ref"
[ -f "$REF/bert.cpp" ] || { echo "build_ref: $REF/bert.cpp not found; skipping"; exit 0; }
TMP="$(mktemp -d)"
trap 'rm -rf "$TMP"' EXIT
sed -n '57,64p'   "$REF/bert.cpp" > "$TMP/vocab_struct.inc"
sed -n '121,134p' "$REF/bert.cpp" > "$TMP/id_to_token.inc"
sed -n '195,417p' "$REF/bert.cpp" > "$TMP/tokenizer.inc"
sed -n '483,493p' "$REF/bert.cpp" > "$TMP/vocab_insert.inc"
# sanity: the ranges must still be what the harness expects
grep -q 'struct bert_vocab' "$TMP/vocab_struct.inc"
grep -q 'bert_vocab_id_to_token' "$TMP/id_to_token.inc"
grep -q 'void bert_tokenize' "$TMP/tokenizer.inc"
grep -q 'subword_token_to_id\[word.substr(2)\]' "$TMP/vocab_insert.inc"
mkdir -p "$OUT"
g++ -O2 -std=c++20 -fPIC -shared -w -I"$REF" -I"$TMP" \
    -o "$OUT/libreftok.so" "$HERE/ref_tokenizer_harness.cpp"
echo "built $OUT/libreftok.so"
