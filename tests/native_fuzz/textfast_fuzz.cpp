// Randomised differential test of the native chunker (docagents_amd/native/textfast.cpp) against a
// plain std::string reference of the same rules (internal/chunker/chunker.go:22-57): random byte
// strings (whitespace, UTF-8 lead bytes, NULs), random / extreme window parameters, undersized
// output buffers. Built with -fsanitize=address,undefined by tests/test_native_sanitized.py, so an
// out-of-bounds access or signed overflow aborts the run. Exit status 0 = every case matched.
#include <climits>
#include <cstdio>
#include <random>
#include <string>
#include <vector>

#include "textfast.cpp"

static bool ws(unsigned char c) { return is_ws(c); }

static std::vector<std::string> ref_chunks(const std::string& s, long maxt, long ov, std::vector<long>& toks) {
  std::vector<std::string> w;
  size_t i = 0;
  while (i < s.size()) {
    while (i < s.size() && ws((unsigned char)s[i])) ++i;
    if (i >= s.size()) break;
    size_t a = i;
    while (i < s.size() && !ws((unsigned char)s[i])) ++i;
    w.push_back(s.substr(a, i - a));
  }
  if (maxt <= 0) maxt = 400;
  if (ov < 0) ov = 0;
  long step = maxt - ov;
  if (step <= 0) step = maxt;
  std::vector<std::string> out;
  const long nw = (long)w.size();
  for (long st = 0; st < nw; st += step) {
    long en = maxt < nw - st ? st + maxt : nw;
    std::string c;
    for (long k = st; k < en; ++k) {
      if (k > st) c += ' ';
      c += w[k];
    }
    out.push_back(c);
    toks.push_back(en - st);
    if (en == nw) break;
  }
  return out;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  std::mt19937_64 rng(12345);
  const char alphabet[] = {'a', 'b', ' ', ' ', '\t', '\n', '\r', '\v', '\f', 'x', '\0', (char)0xc3, (char)0xa0,
                           (char)0x85, (char)0x1c, 'Z', '.', '-'};
  const long extremes[] = {LONG_MIN, -7, -1, 0, 1, 2, 3, 4, 5, 17, 400, 80, LONG_MAX - 1, LONG_MAX};
  long bad = 0;
  for (int it = 0; it < iters; ++it) {
    std::string s(rng() % 300, 'a');
    for (auto& ch : s) ch = alphabet[rng() % sizeof alphabet];
    const long maxt = (rng() & 3) == 0 ? extremes[rng() % 14] : (long)(rng() % 12) - 2;
    const long ov = (rng() & 3) == 0 ? extremes[rng() % 14] : (long)(rng() % 12) - 2;
    // word spans, with an undersized first call (the documented "call again" protocol)
    long cap = (long)(rng() % 4);
    std::vector<int64_t> words(2 * (cap + 1));
    long nw = da_word_offsets(s.data(), (long)s.size(), words.data(), cap);
    if (nw > cap) {
      words.assign(2 * nw + 2, 0);
      if (da_word_offsets(s.data(), (long)s.size(), words.data(), nw) != nw) { ++bad; continue; }
    }
    std::vector<long> toks;
    auto ref = ref_chunks(s, maxt, ov, toks);
    size_t need = 0;
    for (auto& c : ref) need += c.size();
    // out buffer: sometimes too small (must return -1, never write past it)
    const long out_cap = (rng() & 7) == 0 ? (long)(rng() % (need + 2)) : (long)need + 2 * nw + 8;
    const long meta_cap = (rng() & 7) == 0 ? (long)(rng() % (ref.size() + 1)) : (long)ref.size() + 1;
    std::vector<char> out((size_t)out_cap + 1);
    std::vector<int64_t> meta(3 * (size_t)meta_cap + 3);
    if (nw > 0 && (rng() & 15) == 0) {
      // malformed spans: one word's end past the input (or reversed): must be refused
      // with -2 before any byte is copied from past the string (ASan would flag the read)
      std::vector<int64_t> badw(words);
      const long k = (long)(rng() % (unsigned long)nw);
      if (rng() & 1) badw[2 * k + 1] = (int64_t)s.size() + 1 + (int64_t)(rng() % 4096);
      else badw[2 * k] = badw[2 * k + 1] + 1;
      std::vector<char> o2((size_t)s.size() * 8 + 4096);
      std::vector<int64_t> m2(3 * (size_t)nw + 6);
      const long r2 = da_chunk(s.data(), (long)s.size(), badw.data(), nw, maxt, ov, o2.data(), (long)o2.size() - 1,
                               m2.data(), nw + 1);
      if (r2 != -2 && r2 != -1) ++bad;
    }
    long nc = da_chunk(s.data(), (long)s.size(), words.data(), nw, maxt, ov, out.data(), out_cap, meta.data(),
                       meta_cap);
    if (nc == -1) continue;  // undersized buffers: reported, nothing written past them (ASan checks)
    if (nc != (long)ref.size()) { ++bad; continue; }
    for (long c = 0; c < nc; ++c) {
      std::string got(out.data() + meta[3 * c], (size_t)meta[3 * c + 1]);
      if (got != ref[c] || meta[3 * c + 2] != toks[c]) { ++bad; break; }
    }
  }
  printf("{\"iters\": %d, \"mismatches\": %ld}\n", iters, bad);
  return bad ? 1 : 0;
}
