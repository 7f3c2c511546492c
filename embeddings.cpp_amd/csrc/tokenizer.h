// WordPiece tokenizer of the reference (bert.cpp:195-417), re-implemented for
// throughput: byte tries replace the O(len^2) std::map substring probes, the
// text is normalised in one pass, and inputs tokenize in parallel.  Token ids
// are bit-exact with the reference (tests/test_tokenizer.py).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace emb {

class Vocab {
public:
    // Builds the two lookup maps exactly as the loader fills them
    // (bert.cpp:475-494): token_to_id keeps the FIRST id of each string;
    // subword_token_to_id["x"] for every "##x" entry keeps the LAST id.
    void build(const std::vector<std::string> &tokens);

    // bert_tokenize semantics.  Every id is counted in the return value; only
    // the first `cap` are stored.
    int32_t tokenize(const char *text, int32_t n_max_tokens, int32_t *out, int32_t cap) const;

    // bert_vocab_id_to_token semantics (bert.cpp:121-134).
    const char *id_to_token(int32_t id) const;

    size_t size() const { return tokens_.size(); }

private:
    struct Trie {
        // construction: node -> (byte -> child) in a flat open-addressing table
        std::vector<uint64_t> keys;   // (node << 8 | byte) + 1, 0 = empty
        std::vector<int32_t> child;
        std::vector<int32_t> term;    // node -> token id or -1
        int32_t n_nodes = 1;
        void init(size_t expected);
        int32_t add_child(int32_t node, uint8_t b);
        // stores id at the key unless one is there and !overwrite; true if stored
        bool insert(const char *s, size_t n, int32_t id, bool overwrite);
        // lookups: freeze() turns the trie into a double array (base/check, one
        // 8-byte slot per node, nodes placed in breadth-first order so the hot
        // upper levels share cache lines): a step is slot[base[s] + byte] with
        // check == s, one memory access; slots holding a token carry a flag bit
        // and their id sits in a side array.  The construction table's hash
        // probes cost one DRAM miss per byte on a 30k-entry vocab.
        struct Slot { int32_t base; int32_t check; };   // base | kTerm if the slot ends a token
        static constexpr int32_t kTerm = 1 << 30;
        std::vector<Slot> da;         // da[0] = root
        std::vector<int32_t> da_term; // slot -> token id (where flagged)
        void freeze();
        // length of the longest key that is a prefix of s[0..n), 0 if none
        size_t longest(const char *s, size_t n, int32_t *id) const;
    };
    Trie whole_, sub_;
    std::vector<std::string> tokens_;
    std::vector<uint8_t> has_whole_, has_sub_;
};

}  // namespace emb
