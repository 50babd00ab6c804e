// Native text fast path: word spans for the sliding-window chunker (ASCII input).
// Semantics identical to docagents_amd/text/chunker.py (internal/chunker/chunker.go:22-57):
// tokens are maximal runs of non-whitespace; windows of max_tokens words with stride
// max_tokens - overlap; the last window ends at the last word.
#include <stdint.h>
#include <string.h>

// Go's unicode.IsSpace over ASCII (the only input this path takes): exactly these six. Not
// U+001C..U+001F (Python's str.split() cuts there, strings.Fields does not); 0x85 / 0xA0 are
// not ASCII (and as single bytes of UTF-8 text they are continuation bytes, never whitespace).
static inline bool is_ws(unsigned char c) {
  return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f';
}

extern "C" {

// Writes word [start, end) byte offsets into `words` (2 ints per word, capacity cap words).
// Returns the number of words (may exceed cap: call again with a larger buffer).
long da_word_offsets(const char* s, long n, int64_t* words, long cap) {
  long w = 0, i = 0;
  while (i < n) {
    while (i < n && is_ws((unsigned char)s[i])) ++i;
    if (i >= n) break;
    long a = i;
    while (i < n && !is_ws((unsigned char)s[i])) ++i;
    if (w < cap) {
      words[2 * w] = a;
      words[2 * w + 1] = i;
    }
    ++w;
  }
  return w;
}

// Builds all chunk texts (words joined by one space) into `out` (capacity out_cap bytes) and
// writes per chunk [byte_off, byte_len, token_count] into `meta` (3 int64 per chunk).
// Returns the number of chunks, -1 if out/meta are too small, -2 on malformed word spans.
long da_chunk(const char* s, long n, const int64_t* words, long nw, long max_tokens, long overlap, char* out,
              long out_cap, int64_t* meta, long meta_cap) {
  if (max_tokens <= 0) max_tokens = 400;
  if (overlap < 0) overlap = 0;
  if (nw == 0) return 0;
  long step = max_tokens - overlap;
  if (step <= 0) step = max_tokens;
  long nc = 0, o = 0;
  for (long start = 0; start < nw; start += step) {
    // (no start + max_tokens: it overflows for a huge max_tokens)
    long end = max_tokens < nw - start ? start + max_tokens : nw;
    if (nc >= meta_cap) return -1;
    long off = o;
    for (long k = start; k < end; ++k) {
      long len = words[2 * k + 1] - words[2 * k];
      // not spans of s from da_word_offsets (negative, reversed or past the n input bytes)
      if (len < 0 || words[2 * k] < 0 || words[2 * k + 1] > n) return -2;
      if (len > out_cap - o - 1) return -1;
      if (k > start) out[o++] = ' ';
      memcpy(out + o, s + words[2 * k], (size_t)len);
      o += len;
    }
    meta[3 * nc] = off;
    meta[3 * nc + 1] = o - off;
    meta[3 * nc + 2] = end - start;
    ++nc;
    if (end == nw) break;
  }
  return nc;
}
}
