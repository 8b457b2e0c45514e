// Host-side self-test of the C++ runtime (csrc/runtime), built by tests/test_sanitizers_cpu.py with
// -fsanitize=address,undefined (the GPU pool has no device sanitizer; SURVEY §5 asks for ASan/UBSan on
// host code). Each sub-command exercises one component on fixtures the pytest writes:
//   tok  <tokenizer.json> <texts.txt>   encode each line (add_special=1), print ids; decode round-trip
//   fuzz <tokenizer.json> <seed> <n>    random (often invalid UTF-8) byte strings through encode/decode
//   st   <file.safetensors>             every tensor: shape, byte checksum; row/col slices
//   faiss <index> <out>                 read an IxF2 file and write it back
//   bm   <seed>                         randomized BlockManager ops with invariant checks
//   json                                malformed JSON must throw, never crash
//   tokmt <tokenizer.json> <texts.txt>  encode_batch on 8 threads == sequential encode (TSan build: races)
#include <cstdio>
#include <cstring>
#include <fstream>
#include <random>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

#include "json.h"
#include "runtime.h"
#include "tokenizer.h"

using namespace ragk_rt;

static int fail(const char* what) {
  std::fprintf(stderr, "FAIL: %s\n", what);
  return 1;
}

static int cmd_tok(const char* tj, const char* texts) {
  Tokenizer t(tj);
  std::ifstream f(texts);
  std::string line;
  while (std::getline(f, line)) {
    std::vector<int> ids = t.encode(line, true);
    for (size_t i = 0; i < ids.size(); ++i) std::printf(i ? " %d" : "%d", ids[i]);
    std::printf("\n");
    std::string back = t.decode(ids, true);
    std::vector<int> again = t.encode(back, false);  // exercise decode output through encode again
    (void)again;
  }
  return 0;
}

static int cmd_tokmt(const char* tj, const char* texts) {
  Tokenizer t(tj);
  std::ifstream f(texts);
  std::vector<std::string> lines;
  std::string line;
  while (std::getline(f, line)) lines.push_back(line);
  std::vector<std::string> many;
  for (int r = 0; r < 20; ++r)
    for (auto& l : lines) many.push_back(l + " " + std::to_string(r));
  for (int rep = 0; rep < 3; ++rep) {  // cold and warm shared word cache
    std::vector<std::vector<int>> par = t.encode_batch(many, true, 8);
    for (size_t i = 0; i < many.size(); ++i)
      if (par[i] != t.encode(many[i], true)) return fail("encode_batch differs from encode");
  }
  std::printf("tokmt ok %zu\n", many.size());
  return 0;
}

static int cmd_fuzz(const char* tj, unsigned seed, int n) {
  Tokenizer t(tj);
  std::mt19937 rng(seed);
  for (int it = 0; it < n; ++it) {
    std::string s;
    const int len = rng() % 200;
    for (int i = 0; i < len; ++i) {
      const unsigned r = rng() % 10;
      if (r < 5) s.push_back((char)('a' + rng() % 26));
      else if (r < 7) s.push_back(' ');
      else s.push_back((char)(rng() & 0xff));  // arbitrary bytes incl. invalid UTF-8
    }
    std::vector<int> ids = t.encode(s, (it & 1) != 0);
    for (int id : ids)
      if (id < 0 || id >= t.vocab_size()) return fail("token id out of range");
    (void)t.decode(ids, (it & 2) != 0);
    std::vector<int> bad = {0, t.vocab_size() - 1, 1, 2};
    (void)t.decode(bad, false);
  }
  std::printf("fuzz ok %d\n", n);
  return 0;
}

static int cmd_st(const char* path) {
  SafeTensors st(path);
  for (const std::string& k : st.keys()) {
    const TensorInfo& ti = st.info(k);
    unsigned long long sum = 0;
    const unsigned char* p = (const unsigned char*)st.data(k);
    for (size_t i = 0; i < ti.end - ti.begin; ++i) sum = sum * 131 + p[i];
    std::printf("%s %s", k.c_str(), ti.dtype.c_str());
    for (int64_t d : ti.shape) std::printf(" %lld", (long long)d);
    std::printf(" %llu\n", sum);
    if (ti.shape.size() == 2 && ti.shape[0] >= 2 && ti.shape[1] >= 2) {
      const int64_t r1 = ti.shape[0] - 1, c1 = ti.shape[1] - 1;
      std::vector<char> buf((size_t)(r1 - 1) * (c1 - 1) * dtype_size(ti.dtype));
      st.copy_slice(k, 1, r1, 1, c1, buf.data());
      const size_t es = dtype_size(ti.dtype), rb = ti.shape[1] * es;
      for (int64_t r = 1; r < r1; ++r)
        if (std::memcmp(buf.data() + (r - 1) * (c1 - 1) * es, p + r * rb + es, (c1 - 1) * es))
          return fail("slice mismatch");
    }
  }
  bool threw = false;
  try {
    st.info("definitely-not-a-tensor");
  } catch (const std::exception&) {
    threw = true;
  }
  return threw ? 0 : fail("missing tensor must throw");
}

static int cmd_faiss(const char* in, const char* out) {
  FlatIndexData d = read_flat_index(in);
  write_flat_index(out, d.xb.data(), d.ntotal, d.d);
  std::printf("%d %lld\n", d.d, (long long)d.ntotal);
  return 0;
}

static int cmd_bm(unsigned seed) {
  BlockManager bm(40, true);
  std::mt19937 rng(seed);
  std::set<long long> live;
  for (int step = 0; step < 5000; ++step) {
    if (!live.empty() && rng() % 5 < 2) {
      auto it = live.begin();
      std::advance(it, rng() % live.size());
      bm.free(*it);
      live.erase(it);
    } else {
      const long long s = rng() % 12;
      const long long n = 1 + rng() % 600;
      if (bm.can_allocate(s, n)) {
        bm.ensure(s, n);
        live.insert(s);
      }
    }
    std::set<int> used;
    size_t total = 0;
    for (long long s : live)
      for (int b : bm.table(s)) {
        if (b == 0) return fail("scratch block handed out");
        used.insert(b);
        ++total;
      }
    if (used.size() != total) return fail("block shared by two sequences");
    if ((int)total + bm.free_blocks() != bm.num_blocks() - 1) return fail("block leak");
  }
  bool threw = false;
  try {
    bm.ensure(999, 1LL << 30);
  } catch (const std::exception&) {
    threw = true;
  }
  std::printf("bm ok\n");
  return threw ? 0 : fail("oversized ensure must throw");
}

static int cmd_json() {
  const char* bad[] = {"{", "[1,2", "{\"a\":}", "\"\\u12\"", "tru", "{\"a\" 1}", "[1,]x", "\"\\ud800\"", "1e999999",
                       "{\"a\":[{\"b\":\"\\u00e9\\n\"}]", "nul", "-", "\"unterminated"};
  int threw = 0;
  for (const char* s : bad) {
    try {
      Json j = parse_json(s);
      (void)j;
    } catch (const std::exception&) {
      ++threw;
    }
  }
  Json ok = parse_json("{\"a\": [1, 2.5, \"x\\u00e9\", true, null, {\"b\": -3}]}");
  if (ok.at("a").arr.size() != 6) return fail("json array");
  std::printf("json threw %d\n", threw);
  return threw >= 9 ? 0 : fail("malformed JSON accepted");
}

int main(int argc, char** argv) {
  if (argc < 2) return fail("usage");
  const std::string c = argv[1];
  try {
    if (c == "tok" && argc == 4) return cmd_tok(argv[2], argv[3]);
    if (c == "tokmt" && argc == 4) return cmd_tokmt(argv[2], argv[3]);
    if (c == "fuzz" && argc == 5) return cmd_fuzz(argv[2], (unsigned)std::stoul(argv[3]), std::stoi(argv[4]));
    if (c == "st" && argc == 3) return cmd_st(argv[2]);
    if (c == "faiss" && argc == 4) return cmd_faiss(argv[2], argv[3]);
    if (c == "bm" && argc == 3) return cmd_bm((unsigned)std::stoul(argv[2]));
    if (c == "json") return cmd_json();
  } catch (const std::exception& e) {
    std::fprintf(stderr, "exception: %s\n", e.what());
    return 2;
  }
  return fail("bad command");
}
