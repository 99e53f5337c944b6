// ivc_huffman.hip — host-side Huffman coding for the symbol streams (HuffmanCoder,
// ivclab/entropy/huffman.py:5-61).  The north star keeps the serial bit-packing on the host;
// the GPU delivers the symbols and their global histogram.  Canonical codes from the
// Huffman code lengths; bits are packed MSB-first into 32-bit words.
//
// The reference builds its tree with the `constriction` wheel (absent here), whose
// tie-breaking between equal weights is unknown: code lengths can differ between the two on
// ties, so bitstreams (and, when the message is not the training distribution, bit counts)
// are not pinned to the reference.
#include <stdint.h>

#include <algorithm>
#include <queue>
#include <vector>

#include "ivc_internal.h"

namespace ivc {

// Huffman code lengths for n weights (all > 0).  Deterministic: equal weights merge in
// index order of their (sub)trees' first leaf.
int huffman_lengths(const double* w, int32_t n, uint8_t* len) {
  if (n <= 0) return 0;
  if (n == 1) {
    len[0] = 1;
    return 0;
  }
  struct Node {
    double w;
    int32_t first;   // smallest leaf index below (tie-break)
    int32_t id;
  };
  auto cmp = [](const Node& a, const Node& b) {
    if (a.w != b.w) return a.w > b.w;
    return a.first > b.first;
  };
  std::priority_queue<Node, std::vector<Node>, decltype(cmp)> pq(cmp);
  std::vector<int32_t> parent(2 * (size_t)n, -1);
  for (int32_t i = 0; i < n; ++i) pq.push(Node{w[i], i, i});
  int32_t next = n;
  while (pq.size() > 1) {
    const Node a = pq.top(); pq.pop();
    const Node b = pq.top(); pq.pop();
    parent[a.id] = next;
    parent[b.id] = next;
    pq.push(Node{a.w + b.w, std::min(a.first, b.first), next});
    ++next;
  }
  // depth of every leaf
  std::vector<int32_t> depth(next, 0);
  for (int32_t v = next - 2; v >= 0; --v) depth[v] = depth[parent[v]] + 1;
  for (int32_t i = 0; i < n; ++i) {
    if (depth[i] > 64) return -1;
    len[i] = (uint8_t)depth[i];
  }
  return 0;
}

struct Canon {
  std::vector<uint64_t> code;        // per symbol
  std::vector<int32_t> sorted;       // symbols ordered by (length, index)
  uint64_t first_code[66] = {};
  int32_t first_index[66] = {};
  int32_t count[66] = {};
  int maxlen = 0;
};

static bool canonical(const uint8_t* len, int32_t n, Canon& c) {
  c.code.assign(n, 0);
  for (int32_t i = 0; i < n; ++i) {
    if (len[i] == 0 || len[i] > 64) return false;
    c.count[len[i]]++;
    c.maxlen = std::max<int>(c.maxlen, len[i]);
  }
  c.sorted.resize(n);
  int32_t idx = 0;
  for (int L = 1; L <= c.maxlen; ++L) {
    c.first_index[L] = idx;
    for (int32_t i = 0; i < n; ++i)
      if (len[i] == L) c.sorted[idx++] = i;
  }
  uint64_t code = 0;
  for (int L = 1; L <= c.maxlen; ++L) {
    c.first_code[L] = code;
    for (int32_t k = 0; k < c.count[L]; ++k) c.code[c.sorted[c.first_index[L] + k]] = code + k;
    code = (code + c.count[L]) << 1;
  }
  return true;
}

int huffman_encode(const int32_t* sym, int64_t n, int32_t lo, const uint8_t* len, int32_t nalpha,
                   uint32_t* words, int64_t cap, int64_t* nbits) {
  Canon c;
  if (!canonical(len, nalpha, c)) return -1;
  int64_t bits = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t s = (int64_t)sym[i] - lo;
    if (s < 0 || s >= nalpha) return -2;
    bits += len[s];
  }
  *nbits = bits;
  const int64_t need = (bits + 31) / 32;
  if (need > cap) return -3;
  for (int64_t i = 0; i < need; ++i) words[i] = 0;
  int64_t pos = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int32_t s = sym[i] - lo;
    const int L = len[s];
    const uint64_t code = c.code[s];
    for (int k = L - 1; k >= 0; --k, ++pos)
      if ((code >> k) & 1u) words[pos >> 5] |= 0x80000000u >> (pos & 31);
  }
  return 0;
}

int huffman_decode(const uint32_t* words, int64_t nwords, int64_t count, int32_t lo,
                   const uint8_t* len, int32_t nalpha, int32_t* out) {
  Canon c;
  if (!canonical(len, nalpha, c)) return -1;
  const int64_t total = nwords * 32;
  int64_t pos = 0;
  for (int64_t i = 0; i < count; ++i) {
    uint64_t code = 0;
    int L = 0;
    for (;;) {
      if (pos >= total) return -4;                     // stream exhausted
      code = (code << 1) | ((words[pos >> 5] >> (31 - (pos & 31))) & 1u);
      ++pos;
      ++L;
      if (L > c.maxlen) return -5;
      if (c.count[L] && code - c.first_code[L] < (uint64_t)c.count[L]) {
        out[i] = c.sorted[c.first_index[L] + (int32_t)(code - c.first_code[L])] + lo;
        break;
      }
    }
  }
  return 0;
}

}  // namespace ivc
