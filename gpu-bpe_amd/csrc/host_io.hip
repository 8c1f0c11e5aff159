// Host-side formats of the path, native: the v3 trie compiler (trie.js:39-98,
// serializeTrie :167-206) and the DXFT .bin writer (export-controller.js:221-248).
// Byte-exact with the reference (pinned by tests/golden/ref_modules.json trie
// cases and the oracle's dxft_bin).

#include "common.h"

#include <algorithm>
#include <cstring>
#include <vector>

namespace {
constexpr uint32_t kTrieMagic = 0x54524945u;   // 'TRIE', trie.js:20
constexpr uint32_t kTrieVersion = 3;          // trie.js:21
constexpr uint32_t kHeader = 28;              // trie.js:23
constexpr uint32_t kInvalid = 0xFFFFFFFFu;    // engine.js:12
constexpr uint32_t kDxftMagic = 0x44584654u;  // 'DXFT', export-controller.js

struct TNode {
    uint32_t token = kInvalid;
    std::vector<std::pair<uint8_t, int32_t>> kids;   // (byte, node), unsorted until flattening
    int32_t find(uint8_t c) const {
        for (const auto& k : kids)
            if (k.first == c) return k.second;
        return -1;
    }
};

inline void put32(uint8_t* p, uint32_t v) { memcpy(p, &v, 4); }   // little-endian host (x86-64)
}  // namespace

extern "C" int gbpe_trie_compile(const uint8_t* bytes, const uint64_t* offsets, uint32_t n_tokens, uint8_t* out,
                                 uint64_t cap, uint64_t* out_len) {
    if (!out_len || (n_tokens && (!offsets || !bytes))) return GBPE_E_INVALID;
    // 1. tree: token ids in order, a later duplicate overwrites (trie.js:44-57)
    std::vector<TNode> tree(1);
    uint32_t max_len = 0;
    for (uint32_t id = 0; id < n_tokens; ++id) {
        const uint64_t a = offsets[id], b = offsets[id + 1];
        if (b <= a) continue;   // empty entry: skipped (trie.js:46)
        int32_t u = 0;
        for (uint64_t k = a; k < b; ++k) {
            const uint8_t c = bytes[k];
            int32_t v = tree[u].find(c);
            if (v < 0) {
                v = (int32_t)tree.size();
                tree[u].kids.emplace_back(c, v);
                tree.emplace_back();
            }
            u = v;
        }
        tree[u].token = id;
        max_len = std::max<uint32_t>(max_len, (uint32_t)(b - a));
    }
    // 2. BFS flatten, children by byte (trie.js:60-94)
    const uint64_t nn = tree.size(), ne = nn - 1;
    const uint64_t need = kHeader + nn * 12 + ne * 8;
    *out_len = need;
    if (!out) return GBPE_OK;
    if (cap < need) return GBPE_E_CAPACITY;
    std::vector<int32_t> queue;
    queue.reserve(nn);
    queue.push_back(0);
    uint8_t* nodes = out + kHeader;
    uint8_t* edges = nodes + nn * 12;
    uint32_t n_edges = 0;
    for (size_t h = 0; h < queue.size(); ++h) {
        TNode& t = tree[queue[h]];
        std::sort(t.kids.begin(), t.kids.end());
        const uint32_t first = n_edges;
        uint32_t num = 0;
        for (const auto& k : t.kids) {
            const uint32_t idx = (uint32_t)queue.size();
            queue.push_back(k.second);
            uint8_t* e = edges + (uint64_t)n_edges * 8;
            e[0] = k.first;
            e[1] = e[2] = e[3] = 0;
            put32(e + 4, idx);
            ++n_edges;
            ++num;
        }
        uint8_t* nd = nodes + h * 12;
        put32(nd, first);
        put32(nd + 4, num);
        put32(nd + 8, t.token);
    }
    // 3. header (serializeTrie, trie.js:178-184)
    put32(out, kTrieMagic);
    put32(out + 4, kTrieVersion);
    put32(out + 8, (uint32_t)nn);
    put32(out + 12, n_edges);
    put32(out + 16, max_len);
    put32(out + 20, n_tokens);
    put32(out + 24, 0);
    return GBPE_OK;
}

extern "C" int gbpe_dxft_pack(const uint32_t* tokens, uint64_t n_tokens, uint32_t vocab_size, const uint8_t* vocab_json,
                              uint64_t json_len, uint8_t* out, uint64_t cap, uint64_t* out_len) {
    if (!out_len || (n_tokens && !tokens) || (json_len && !vocab_json)) return GBPE_E_INVALID;
    const uint64_t need = 16 + 4 * n_tokens + json_len;
    *out_len = need;
    if (!out) return GBPE_OK;
    if (cap < need) return GBPE_E_CAPACITY;
    put32(out, kDxftMagic);
    put32(out + 4, vocab_size);
    put32(out + 8, (uint32_t)n_tokens);
    put32(out + 12, (uint32_t)json_len);
    if (n_tokens) memcpy(out + 16, tokens, 4 * n_tokens);
    if (json_len) memcpy(out + 16 + 4 * n_tokens, vocab_json, json_len);
    return GBPE_OK;
}
