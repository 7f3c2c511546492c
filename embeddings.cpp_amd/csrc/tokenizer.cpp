// Fast bit-exact WordPiece (see tokenizer.h).  Character classes are the
// C-locale ASCII ones the reference sees through ispunct/isspace on plain
// `char` (bytes >= 0x80 are never punctuation or space there).
#include "tokenizer.h"

#include <algorithm>
#include <cstring>
#include <vector>
#include <utility>

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
    n_nodes = 1;
}

int32_t Vocab::Trie::add_child(int32_t node, uint8_t b)
{
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
            return n_nodes++;
        }
        if (keys[i] == k) return child[i];
        i = (i + 1) & (keys.size() - 1);
    }
}

bool Vocab::Trie::insert(const char *s, size_t n, int32_t id, bool overwrite)
{
    int32_t node = 0;
    for (size_t i = 0; i < n; ++i) node = add_child(node, (uint8_t)s[i]);
    if (term[(size_t)node] < 0 || overwrite) {
        term[(size_t)node] = id;
        return true;
    }
    return false;
}

void Vocab::Trie::freeze()
{
    const size_t N = (size_t)n_nodes;
    // the edges grouped by parent (counting sort), bytes ascending within a parent
    std::vector<int32_t> cnt(N + 1, 0);
    for (size_t j = 0; j < keys.size(); ++j)
        if (keys[j]) ++cnt[(size_t)((keys[j] - 1) >> 8) + 1];
    for (size_t v = 0; v < N; ++v) cnt[v + 1] += cnt[v];
    std::vector<std::pair<uint8_t, int32_t>> adj((size_t)cnt[N]);
    std::vector<int32_t> fill(cnt.begin(), cnt.end() - 1);
    for (size_t j = 0; j < keys.size(); ++j)
        if (keys[j]) {
            const size_t p = (size_t)((keys[j] - 1) >> 8);
            adj[(size_t)fill[p]++] = {(uint8_t)((keys[j] - 1) & 0xff), child[j]};
        }
    for (size_t v = 0; v < N; ++v) std::sort(adj.begin() + cnt[v], adj.begin() + cnt[v + 1]);
    // double array, nodes placed breadth-first: each node's children go to the
    // first base b with every slot b + byte free (first-fit from the lowest free
    // slot); slot 0 is the root, check = parent slot, -1 = free
    std::vector<int32_t> pos(N, -1);   // node -> slot
    da.assign(N + 512, Slot{0, -1});
    std::vector<int32_t> sterm(da.size(), -1);
    std::vector<uint8_t> used(da.size(), 0), base_used(da.size(), 0);
    auto ensure = [&](size_t n) {
        if (n > da.size()) {
            const size_t m = std::max(n, da.size() * 3 / 2);
            da.resize(m, Slot{0, -1});
            sterm.resize(m, -1);
            used.resize(m, 0);
            base_used.resize(m, 0);
        }
    };
    pos[0] = 0;
    used[0] = 1;
    da[0].check = 0;
    size_t first_free = 1;
    std::vector<int32_t> queue;
    queue.reserve(N);
    queue.push_back(0);
    for (size_t h = 0; h < queue.size(); ++h) {
        const int32_t v = queue[h];
        const int32_t sv = pos[(size_t)v];
        sterm[(size_t)sv] = term[(size_t)v];
        const int32_t e0 = cnt[(size_t)v], e1 = cnt[(size_t)v + 1];
        if (e0 == e1) continue;
        while (first_free < used.size() && used[first_free]) ++first_free;
        const int32_t c0 = adj[(size_t)e0].first;
        // base candidates: the first child lands on a free slot at or past first_free
        for (int64_t b = std::max<int64_t>(1, (int64_t)first_free - c0);; ++b) {
            ensure((size_t)b + 256);
            if (base_used[(size_t)b] || used[(size_t)(b + c0)]) continue;
            bool ok = true;
            for (int32_t e = e0 + 1; e < e1 && ok; ++e) ok = !used[(size_t)(b + adj[(size_t)e].first)];
            if (!ok) continue;
            base_used[(size_t)b] = 1;      // distinct bases: a slot's check names one parent
            da[(size_t)sv].base = (int32_t)b;
            for (int32_t e = e0; e < e1; ++e) {
                const size_t slot = (size_t)(b + adj[(size_t)e].first);
                used[slot] = 1;
                da[slot].check = sv;
                pos[(size_t)adj[(size_t)e].second] = (int32_t)slot;
                queue.push_back(adj[(size_t)e].second);
            }
            break;
        }
    }
    size_t last = 0;
    for (size_t i = 0; i < used.size(); ++i)
        if (used[i]) last = i;
    da.resize(last + 257, Slot{0, -1});   // every base + byte stays in range
    sterm.resize(da.size(), -1);
    for (size_t i = 0; i < da.size(); ++i)
        if (sterm[i] >= 0) da[i].base |= kTerm;
    da_term.swap(sterm);
    std::vector<uint64_t>().swap(keys);
    std::vector<int32_t>().swap(child);
    std::vector<int32_t>().swap(term);
}

size_t Vocab::Trie::longest(const char *s, size_t n, int32_t *id) const
{
    const Slot *d = da.data();
    int32_t cur = 0, base = d[0].base & ~kTerm;
    size_t best = 0;
    for (size_t i = 0; i < n; ++i) {
        const int32_t nx = base + (uint8_t)s[i];
        if (d[nx].check != cur || nx == 0) break;
        cur = nx;
        base = d[cur].base;
        if (base & kTerm) { best = i + 1; base &= ~kTerm; *id = da_term[(size_t)cur]; }
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
        // first occurrence wins; the empty string is a key too (never looked up)
        if (w.empty()) {
            if (!empty_seen) { has_whole_[i] = 1; empty_seen = true; }
            continue;
        }
        if (whole_.insert(w.data(), w.size(), (int32_t)i, false)) has_whole_[i] = 1;
    }
    whole_.freeze();
    sub_.freeze();
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

    // 1) accent strip + A-Z lowercase at character starts (bert.cpp:206-251), one
    // pass: a character's first byte is the only place an ASCII letter can be
    // lowered (bytes inside a malformed multi-byte span are copied raw, as the
    // reference's char-stride loop leaves them); per-thread scratch buffers
    thread_local std::vector<char> abuf, bbuf;
    if (abuf.size() < n_in + 1) abuf.resize(n_in + 1);
    char *a = abuf.data();
    size_t na = 0;
    for (size_t i = 0; i < n_in;) {
        const uint8_t c = in[i];
        if (c < 0x80) {
            a[na++] = (char)(c >= 'A' && c <= 'Z' ? c - 'A' + 'a' : c);
            ++i;
            continue;
        }
        const size_t len = (size_t)lead_len(c);
        const size_t take = i + len <= n_in ? len : n_in - i;
        if (take == 2 && c == 0xC3 && kAccents.map[in[i + 1]]) {
            const char m = kAccents.map[in[i + 1]];
            a[na++] = (char)(m >= 'A' && m <= 'Z' ? m - 'A' + 'a' : m);
        } else {
            for (size_t k = 0; k < take; ++k) a[na++] = (char)in[i + k];
        }
        i += take;
    }

    // 2) isolate ASCII punctuation and 3-byte CJK (bert.cpp:317-339), byte by
    // byte over the normalised text as the reference walks it
    if (bbuf.size() < 3 * na + 8) bbuf.resize(3 * na + 8);
    char *b = bbuf.data();
    size_t nbb = 0;
    const uint8_t *pa = (const uint8_t *)a;
    for (size_t i = 0; i < na;) {
        const uint8_t c = pa[i];
        if (c < 0x80) {
            if (is_punct(c)) { b[nbb] = ' '; b[nbb + 1] = (char)c; b[nbb + 2] = ' '; nbb += 3; }
            else b[nbb++] = (char)c;
            ++i;
        } else if (lead_len(c) == 3 && is_cjk3(pa + i, na - i)) {
            b[nbb] = ' '; b[nbb + 1] = (char)c; b[nbb + 2] = (char)pa[i + 1]; b[nbb + 3] = (char)pa[i + 2];
            b[nbb + 4] = ' ';
            nbb += 5;
            i += 3;
        } else {
            b[nbb++] = (char)c;
            ++i;
        }
    }

    // 4) greedy longest-prefix WordPiece per word (bert.cpp:369-416)
    int32_t t = 0;
    auto emit = [&](int32_t id) { if (t < cap) out[t] = id; ++t; };
    emit(101);
    const char *pb = b;
    const size_t nb = nbb;
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
