// Fast bit-exact WordPiece (see tokenizer.h).  Character classes are the
// C-locale ASCII ones the reference sees through ispunct/isspace on plain
// `char` (bytes >= 0x80 are never punctuation or space there).
#include "tokenizer.h"

#include <cstring>

namespace emb {

namespace {

inline int lead_len(uint8_t c)
{
    // utf8_len (bert.cpp:199-204): decided by the high nibble of the byte
    return c < 0xC0 ? 1 : (c < 0xE0 ? 2 : (c < 0xF0 ? 3 : 4));
}

inline bool is_punct(uint8_t c)
{
    return (c >= 0x21 && c <= 0x2F) || (c >= 0x3A && c <= 0x40) || (c >= 0x5B && c <= 0x60) || (c >= 0x7B && c <= 0x7E);
}

inline bool is_space(uint8_t c) { return c == 0x20 || (c >= 0x09 && c <= 0x0D); }

// stripAccents (bert.cpp:206-238): 52 Latin-1 letters, all encoded C3 xx.
// Index by the second byte; 0 = leave unchanged.
struct AccentTable {
    char map[256];
    AccentTable()
    {
        std::memset(map, 0, sizeof(map));
        const char *up = "AAAAAA.CEEEEIIII.NOOOOO..UUUUY";   // C3 80 .. C3 9D
        for (int i = 0; up[i]; ++i) {
            if (up[i] == '.') continue;
            map[0x80 + i] = up[i];
            map[0xA0 + i] = (char)(up[i] - 'A' + 'a');     // C3 A0 .. C3 BD
        }
    }
};
const AccentTable kAccents;

// is_Chinese_char (bert.cpp:253-295) for a well-formed 3-byte sequence.  The
// reference's 4-byte ranges are unreachable: it only asks for 3-byte leads.
inline bool is_cjk3(const uint8_t *p, size_t avail)
{
    if (avail < 3 || (p[1] & 0xC0) != 0x80 || (p[2] & 0xC0) != 0x80) return false;
    const uint32_t cp = ((uint32_t)(p[0] & 0x0F) << 12) | ((uint32_t)(p[1] & 0x3F) << 6) | (p[2] & 0x3F);
    return (cp >= 0x4E00 && cp <= 0x9FFF) || (cp >= 0x3400 && cp <= 0x4DBF) || (cp >= 0xF900 && cp <= 0xFAFF) ||
           (cp >= 0x3000 && cp <= 0x303F) || (cp >= 0xFF00 && cp <= 0xFFEF);
}

inline uint64_t mix(uint64_t k)
{
    k ^= k >> 33; k *= 0xff51afd7ed558ccdULL; k ^= k >> 33;
    return k;
}

}  // namespace

void Vocab::Trie::init(size_t expected)
{
    size_t cap = 1024;
    while (cap < expected * 4) cap <<= 1;
    keys.assign(cap, 0);
    child.assign(cap, 0);
    term.assign(1, -1);
    for (int32_t &r : root) r = -1;
    n_nodes = 1;
}

int32_t Vocab::Trie::step(int32_t node, uint8_t b) const
{
    const uint64_t k = (((uint64_t)node << 8) | b) + 1;
    size_t i = mix(k) & (keys.size() - 1);
    for (;;) {
        if (keys[i] == 0) return -1;
        if (keys[i] == k) return child[i];
        i = (i + 1) & (keys.size() - 1);
    }
}

int32_t Vocab::Trie::add_child(int32_t node, uint8_t b)
{
    if (node == 0 && root[b] >= 0) return root[b];
    const uint64_t k = (((uint64_t)node << 8) | b) + 1;
    if ((size_t)n_nodes * 2 >= keys.size()) {     // grow
        std::vector<uint64_t> ok;
        std::vector<int32_t> oc;
        ok.swap(keys);
        oc.swap(child);
        keys.assign(ok.size() * 2, 0);
        child.assign(ok.size() * 2, 0);
        for (size_t j = 0; j < ok.size(); ++j) {
            if (!ok[j]) continue;
            size_t i = mix(ok[j]) & (keys.size() - 1);
            while (keys[i]) i = (i + 1) & (keys.size() - 1);
            keys[i] = ok[j];
            child[i] = oc[j];
        }
    }
    size_t i = mix(k) & (keys.size() - 1);
    for (;;) {
        if (keys[i] == 0) {
            keys[i] = k;
            child[i] = n_nodes;
            term.push_back(-1);
            if (node == 0) root[b] = n_nodes;
            return n_nodes++;
        }
        if (keys[i] == k) return child[i];
        i = (i + 1) & (keys.size() - 1);
    }
}

void Vocab::Trie::insert(const char *s, size_t n, int32_t id, bool overwrite)
{
    int32_t node = 0;
    for (size_t i = 0; i < n; ++i) node = add_child(node, (uint8_t)s[i]);
    if (term[(size_t)node] < 0 || overwrite) term[(size_t)node] = id;
}

size_t Vocab::Trie::longest(const char *s, size_t n, int32_t *id) const
{
    if (n == 0) return 0;
    int32_t node = root[(uint8_t)s[0]];
    if (node < 0) return 0;
    size_t best = 0;
    if (term[(size_t)node] >= 0) { best = 1; *id = term[(size_t)node]; }
    for (size_t i = 1; i < n; ++i) {
        node = step(node, (uint8_t)s[i]);
        if (node < 0) break;
        if (term[(size_t)node] >= 0) { best = i + 1; *id = term[(size_t)node]; }
    }
    return best;
}

void Vocab::build(const std::vector<std::string> &tokens)
{
    tokens_ = tokens;
    has_whole_.assign(tokens.size(), 0);
    has_sub_.assign(tokens.size(), 0);
    whole_.init(tokens.size() * 8);
    sub_.init(tokens.size() * 8);
    bool empty_seen = false;
    for (size_t i = 0; i < tokens.size(); ++i) {
        const std::string &w = tokens[i];
        if (w.size() >= 2 && w[0] == '#' && w[1] == '#') {
            sub_.insert(w.data() + 2, w.size() - 2, (int32_t)i, /*overwrite=*/true);
            has_sub_[i] = 1;
        }
        int32_t tmp;
        // first occurrence wins; the empty string is a key too (never looked up)
        if (w.empty()) {
            if (!empty_seen) { has_whole_[i] = 1; empty_seen = true; }
            continue;
        }
        if (whole_.longest(w.data(), w.size(), &tmp) != w.size()) {
            whole_.insert(w.data(), w.size(), (int32_t)i, false);
            has_whole_[i] = 1;
        }
    }
}

const char *Vocab::id_to_token(int32_t id) const
{
    if (id >= 0 && (size_t)id < tokens_.size() && (has_whole_[(size_t)id] || has_sub_[(size_t)id]))
        return tokens_[(size_t)id].c_str();
    return "[UNK TOKEN from bert_vocab]";
}

int32_t Vocab::tokenize(const char *text, int32_t n_max_tokens, int32_t *out, int32_t cap) const
{
    const uint8_t *in = (const uint8_t *)text;
    const size_t n_in = std::strlen(text);

    // 1) accent strip + A-Z lowercase at character starts (bert.cpp:206-251);
    // per-thread scratch strings keep their capacity across calls
    thread_local std::string a, b;
    a.clear();
    a.reserve(n_in);
    for (size_t i = 0; i < n_in;) {
        const size_t len = (size_t)lead_len(in[i]);
        const size_t take = i + len <= n_in ? len : n_in - i;
        if (take == 2 && in[i] == 0xC3 && kAccents.map[in[i + 1]]) a.push_back(kAccents.map[in[i + 1]]);
        else a.append((const char *)in + i, take);
        i += take;
    }
    for (size_t i = 0; i < a.size(); i += (size_t)lead_len((uint8_t)a[i]))
        if (a[i] >= 'A' && a[i] <= 'Z') a[i] = (char)(a[i] - 'A' + 'a');

    // 2) isolate ASCII punctuation and 3-byte CJK (bert.cpp:317-339),
    // 3) whitespace split (bert.cpp:341-358) -- fused: collect word spans.
    b.clear();
    b.reserve(a.size() * 2 + 8);
    const uint8_t *pa = (const uint8_t *)a.data();
    for (size_t i = 0; i < a.size();) {
        const int len = lead_len(pa[i]);
        if (len == 1 && is_punct(pa[i])) {
            b.push_back(' '); b.push_back((char)pa[i]); b.push_back(' ');
            i += 1;
        } else if (len == 3 && is_cjk3(pa + i, a.size() - i)) {
            b.push_back(' '); b.append((const char *)pa + i, 3); b.push_back(' ');
            i += 3;
        } else {
            b.push_back((char)pa[i]);
            i += 1;
        }
    }

    // 4) greedy longest-prefix WordPiece per word (bert.cpp:369-416)
    int32_t t = 0;
    auto emit = [&](int32_t id) { if (t < cap) out[t] = id; ++t; };
    emit(101);
    const char *pb = b.data();
    const size_t nb = b.size();
    size_t l = 0;
    for (size_t r = 0; r <= nb; ++r) {
        if (r < nb && !is_space((uint8_t)pb[r])) continue;
        if (r > l) {
            const char *w = pb + l;
            const size_t n = r - l;
            const int32_t prev = t;
            const Trie *map = &whole_;
            size_t i = 0;
            while (i < n) {
                if (t >= n_max_tokens - 1) break;
                int32_t id = -1;
                const size_t m = map->longest(w + i, n - i, &id);
                map = &sub_;
                if (m) { emit(id); i += m; }
                else { ++i; }          // unmatched byte is skipped (bert.cpp:401-406)
            }
            if (prev == t) emit(100);
        }
        l = r + 1;
    }
    emit(102);
    return t;
}

}  // namespace emb
