#include "tokenizer.h"

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <exception>
#include <mutex>
#include <thread>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <limits>
#include <sstream>
#include <stdexcept>

#include "unicode_tables.h"

namespace ragk_rt {

namespace {

bool in_ranges(const CpRange* r, int n, uint32_t c) {
  int lo = 0, hi = n - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    if (c < r[mid].lo) hi = mid - 1;
    else if (c > r[mid].hi) lo = mid + 1;
    else return true;
  }
  return false;
}
uint32_t map_lookup(const uint32_t (*m)[2], int n, uint32_t c) {
  int lo = 0, hi = n - 1;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    if (c < m[mid][0]) hi = mid - 1;
    else if (c > m[mid][0]) lo = mid + 1;
    else return m[mid][1];
  }
  return c;
}
inline bool is_L(uint32_t c) { return c < 0x80 ? ((c | 32) - 'a' < 26u) : in_ranges(UNI_L, UNI_L_N, c); }
inline bool is_N(uint32_t c) { return c < 0x80 ? (c - '0' < 10u) : in_ranges(UNI_N, UNI_N_N, c); }
inline bool is_WS(uint32_t c) { return in_ranges(UNI_WS, UNI_WS_N, c); }
inline bool is_crlf(uint32_t c) { return c == '\r' || c == '\n'; }
inline bool is_bert_punct(uint32_t c) {
  if ((c >= 33 && c <= 47) || (c >= 58 && c <= 64) || (c >= 91 && c <= 96) || (c >= 123 && c <= 126)) return true;
  return in_ranges(UNI_P, UNI_P_N, c);
}
inline bool is_cjk(uint32_t c) {
  return (c >= 0x4E00 && c <= 0x9FFF) || (c >= 0x3400 && c <= 0x4DBF) || (c >= 0x20000 && c <= 0x2A6DF) ||
         (c >= 0x2A700 && c <= 0x2B73F) || (c >= 0x2B740 && c <= 0x2B81F) || (c >= 0x2B820 && c <= 0x2CEAF) ||
         (c >= 0xF900 && c <= 0xFAFF) || (c >= 0x2F800 && c <= 0x2FA1F);
}

// ---- regex pre-tokenizers, hand-matched (alternation order = regex order) ----
// GPT-2: 's|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+
size_t contraction(const std::vector<uint32_t>& c, size_t i, bool icase) {
  if (c[i] != '\'' || i + 1 >= c.size()) return 0;
  auto low = [&](uint32_t x) { return icase && x < 128 ? (uint32_t)tolower((int)x) : x; };
  const uint32_t a = low(c[i + 1]);
  if (a == 's' || a == 't' || a == 'm' || a == 'd') return 2;
  if (i + 2 < c.size()) {
    const uint32_t b = low(c[i + 2]);
    if ((a == 'r' && b == 'e') || (a == 'v' && b == 'e') || (a == 'l' && b == 'l')) return 3;
  }
  return 0;
}
size_t ws_tail(const std::vector<uint32_t>& c, size_t i) {  // \s+(?!\S) then \s+
  size_t j = i;
  while (j < c.size() && is_WS(c[j])) ++j;
  if (j == i) return 0;
  if (j == c.size()) return j - i;
  if (j - i >= 2) return j - i - 1;
  return j - i;
}
size_t match_gpt2(const std::vector<uint32_t>& c, size_t i) {
  const size_t n = c.size();
  if (size_t k = contraction(c, i, false)) return k;
  size_t s = (c[i] == ' ' && i + 1 < n) ? 1 : 0;
  for (int cls = 0; cls < 3; ++cls) {
    for (size_t sp = s; ; sp = 0) {  // try with the optional space, then without
      size_t j = i + sp;
      auto ok = [&](uint32_t x) {
        return cls == 0 ? is_L(x) : cls == 1 ? is_N(x) : (!is_WS(x) && !is_L(x) && !is_N(x));
      };
      if (j < n && ok(c[j])) {
        while (j < n && ok(c[j])) ++j;
        return j - i;
      }
      if (sp == 0) break;
    }
  }
  return ws_tail(c, i);
}
// Llama-3: (?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}| ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+
size_t match_llama3(const std::vector<uint32_t>& c, size_t i) {
  const size_t n = c.size();
  if (size_t k = contraction(c, i, true)) return k;
  {  // [^\r\n\p{L}\p{N}]?\p{L}+
    size_t j = i;
    if (!is_crlf(c[j]) && !is_L(c[j]) && !is_N(c[j]) && j + 1 < n && is_L(c[j + 1])) ++j;
    if (j < n && is_L(c[j])) {
      while (j < n && is_L(c[j])) ++j;
      return j - i;
    }
  }
  if (is_N(c[i])) {  // \p{N}{1,3}
    size_t j = i;
    while (j < n && j - i < 3 && is_N(c[j])) ++j;
    return j - i;
  }
  {  //  ?[^\s\p{L}\p{N}]+[\r\n]*
    auto sym = [&](uint32_t x) { return !is_WS(x) && !is_L(x) && !is_N(x); };
    size_t j = i + ((c[i] == ' ' && i + 1 < n && sym(c[i + 1])) ? 1 : 0);
    if (j < n && sym(c[j])) {
      while (j < n && sym(c[j])) ++j;
      while (j < n && is_crlf(c[j])) ++j;
      return j - i;
    }
  }
  {  // \s*[\r\n]+
    size_t j = i;
    while (j < n && is_WS(c[j])) ++j;
    size_t last = std::string::npos;
    for (size_t k = i; k < j; ++k)
      if (is_crlf(c[k])) last = k;
    if (last != std::string::npos) return last + 1 - i;
  }
  if (size_t k = ws_tail(c, i)) return k;
  return 1;
}

std::string cp_utf8(uint32_t cp) {
  std::string s;
  append_utf8(s, cp);
  return s;
}

}  // namespace

std::vector<uint32_t> utf8_decode(const std::string& s) {
  std::vector<uint32_t> out;
  out.reserve(s.size());
  const unsigned char* p = (const unsigned char*)s.data();
  const size_t n = s.size();
  size_t i = 0;
  while (i < n) {
    const unsigned c = p[i];
    uint32_t cp;
    int len;
    if (c < 0x80) { cp = c; len = 1; }
    else if ((c >> 5) == 6) { cp = c & 0x1F; len = 2; }
    else if ((c >> 4) == 14) { cp = c & 0x0F; len = 3; }
    else if ((c >> 3) == 30) { cp = c & 0x07; len = 4; }
    else { out.push_back(0xFFFD); ++i; continue; }
    if (i + len > n) { out.push_back(0xFFFD); ++i; continue; }
    bool ok = true;
    for (int k = 1; k < len; ++k) {
      if ((p[i + k] >> 6) != 2) { ok = false; break; }
      cp = (cp << 6) | (p[i + k] & 0x3F);
    }
    if (!ok) { out.push_back(0xFFFD); ++i; continue; }
    out.push_back(cp);
    i += len;
  }
  return out;
}

std::string utf8_encode(const std::vector<uint32_t>& cps, size_t b, size_t e) {
  std::string s;
  for (size_t i = b; i < e; ++i) append_utf8(s, cps[i]);
  return s;
}

static unsigned long long g_tok_uid_next() {
  static std::atomic<unsigned long long> c{1};
  return c++;
}

Tokenizer::Tokenizer(const std::string& path) : uid_(g_tok_uid_next()) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  std::stringstream ss;
  ss << f.rdbuf();
  const Json j = parse_json(ss.str());
  // GPT-2 bytes_to_unicode
  std::vector<int> bs;
  for (int b = '!'; b <= '~'; ++b) bs.push_back(b);
  for (int b = 0xA1; b <= 0xAC; ++b) bs.push_back(b);
  for (int b = 0xAE; b <= 0xFF; ++b) bs.push_back(b);
  std::vector<bool> have(256, false);
  for (int b : bs) {
    have[b] = true;
    byte_to_uni_[b] = cp_utf8(b);
    uni_to_byte_[b] = (unsigned char)b;
  }
  int extra = 0;
  for (int b = 0; b < 256; ++b)
    if (!have[b]) {
      byte_to_uni_[b] = cp_utf8(256 + extra);
      uni_to_byte_[256 + extra] = (unsigned char)b;
      ++extra;
    }
  load_model(j.at("model"));
  if (const Json* at = j.get("added_tokens")) {
    for (auto& t : at->arr) {
      Added a{(int)t.at("id").as_int(), t.at("content").str, t.get("special") && t.at("special").truthy()};
      added_.push_back(a);
      if (a.special) special_ids_.insert(a.id);
      if ((int)id_to_tok_.size() <= a.id) id_to_tok_.resize(a.id + 1);
      id_to_tok_[a.id] = a.content;
      vocab_[a.content] = a.id;
      if (!a.content.empty()) added_first_bytes_.insert((unsigned char)a.content[0]);
    }
    std::sort(added_.begin(), added_.end(),
              [](const Added& x, const Added& y) { return x.content.size() > y.content.size(); });
  }
  load_normalizer(j.get("normalizer"));
  load_pre(j.get("pre_tokenizer"));
  load_post(j.get("post_processor"));
  load_decoder(j.get("decoder"));
  slice_safe_ = pre_ == PRE_BERT || pre_ == PRE_WHITESPACE;
  for (const auto& st : norm_) slice_safe_ = slice_safe_ && (st.kind == NormStep::BERT || st.kind == NormStep::LOWER);
}

void Tokenizer::load_model(const Json& m) {
  model_name_ = m.at("type").str;
  auto put = [&](const std::string& t, int id) {
    vocab_[t] = id;
    if ((int)id_to_tok_.size() <= id) id_to_tok_.resize(id + 1);
    id_to_tok_[id] = t;
  };
  if (model_name_ == "BPE") {
    model_ = BPE;
    for (auto& kv : m.at("vocab").obj) put(kv.first, (int)kv.second.as_int());
    if (const Json* im = m.get("ignore_merges")) ignore_merges_ = im->truthy();
    if (const Json* bf = m.get("byte_fallback")) byte_fallback_ = bf->truthy();
    int rank = 0;
    for (auto& mg : m.at("merges").arr) {
      std::string a, b;
      if (mg.type == Json::STR) {
        const size_t sp = mg.str.find(' ', 1);
        if (sp == std::string::npos) { ++rank; continue; }
        a = mg.str.substr(0, sp);
        b = mg.str.substr(sp + 1);
      } else {
        a = mg.arr.at(0).str;
        b = mg.arr.at(1).str;
      }
      auto ia = vocab_.find(a), ib = vocab_.find(b), im = vocab_.find(a + b);
      if (ia != vocab_.end() && ib != vocab_.end() && im != vocab_.end()) {
        const uint64_t key = ((uint64_t)(uint32_t)ia->second << 32) | (uint32_t)ib->second;
        if (!merges_.count(key)) merges_[key] = {rank, im->second};
      }
      ++rank;
    }
  } else if (model_name_ == "WordPiece") {
    model_ = WORDPIECE;
    for (auto& kv : m.at("vocab").obj) put(kv.first, (int)kv.second.as_int());
    if (const Json* u = m.get("unk_token")) unk_token_ = u->str;
    if (const Json* p = m.get("continuing_subword_prefix")) wp_prefix_ = p->str;
    if (const Json* x = m.get("max_input_chars_per_word")) max_chars_per_word_ = (int)x->as_int();
  } else if (model_name_ == "Unigram") {
    model_ = UNIGRAM;
    int id = 0;
    min_score_ = std::numeric_limits<double>::infinity();
    for (auto& e : m.at("vocab").arr) {
      put(e.arr.at(0).str, id);
      scores_.push_back(e.arr.at(1).as_num());
      min_score_ = std::min(min_score_, scores_.back());
      ++id;
    }
    if (const Json* u = m.get("unk_id")) unk_id_ = u->is_null() ? 0 : (int)u->as_int();
  } else {
    throw std::runtime_error("unsupported tokenizer model " + model_name_);
  }
}

static std::string base64_decode(const std::string& in) {
  static int T[256];
  static bool init = false;
  if (!init) {
    for (int i = 0; i < 256; ++i) T[i] = -1;
    const char* a = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
    for (int i = 0; i < 64; ++i) T[(unsigned char)a[i]] = i;
    init = true;
  }
  std::string out;
  uint32_t val = 0;
  int bits = -8;
  for (unsigned char c : in) {
    if (T[c] < 0) continue;  // '=' padding / whitespace
    val = ((val << 6) | (uint32_t)T[c]) & 0xFFFFFFu;  // only the last 24 bits are ever read
    bits += 6;
    if (bits >= 0) {
      out.push_back((char)((val >> bits) & 0xFF));
      bits -= 8;
    }
  }
  return out;
}

void Tokenizer::load_normalizer(const Json* n) {
  if (!n || n->is_null()) return;
  const std::string t = n->at("type").str;
  NormStep st{};
  if (t == "Sequence") {
    for (auto& x : n->at("normalizers").arr) load_normalizer(&x);
    return;
  } else if (t == "BertNormalizer") {
    st.kind = NormStep::BERT;
    if (const Json* x = n->get("clean_text")) bn_clean_ = x->truthy();
    if (const Json* x = n->get("handle_chinese_chars")) bn_chinese_ = x->truthy();
    if (const Json* x = n->get("lowercase")) bn_lower_ = x->truthy();
    const Json* sa = n->get("strip_accents");
    bn_strip_ = (sa && !sa->is_null()) ? sa->truthy() : bn_lower_;
  } else if (t == "Lowercase") {
    st.kind = NormStep::LOWER;
  } else if (t == "Strip") {
    st.kind = NormStep::STRIP;
    if (const Json* x = n->get("strip_left")) st.left = x->truthy();
    if (const Json* x = n->get("strip_right")) st.right = x->truthy();
  } else if (t == "Replace") {
    const Json& pat = n->at("pattern");
    st.content = n->at("content").str;
    if (const Json* lit = pat.get("String")) {
      st.kind = NormStep::REPLACE;
      st.pat = lit->str;
      if (st.pat.empty()) return;
    } else {
      // only single-code-point runs "c{n,}" (the SentencePiece converters' " {2,}")
      const std::string rx = pat.at("Regex").str;
      std::vector<uint32_t> cps = utf8_decode(rx);
      size_t brace = 0;
      while (brace < cps.size() && cps[brace] != '{') ++brace;
      if (brace != 1 || cps.size() < 5 || cps.back() != '}' || cps[cps.size() - 2] != ',')
        throw std::runtime_error("unsupported Replace regex: " + rx);
      st.kind = NormStep::REPLACE_RUN;
      st.run_cp = cps[0];
      st.run_min = std::stoi(utf8_encode(cps, 2, cps.size() - 2));
    }
  } else if (t == "Precompiled") {
    st.kind = NormStep::PRECOMPILED;
    const Json* pc = n->get("precompiled_charsmap");
    const std::string blob = (pc && pc->type == Json::STR) ? base64_decode(pc->str) : std::string();
    if (blob.size() < 4) return;  // empty charsmap = identity
    uint32_t tsz = 0;
    memcpy(&tsz, blob.data(), 4);
    if (tsz % 4 || 4 + (size_t)tsz > blob.size()) throw std::runtime_error("corrupt precompiled_charsmap");
    pc_trie_.resize(tsz / 4);
    memcpy(pc_trie_.data(), blob.data() + 4, tsz);
    pc_norm_ = blob.substr(4 + tsz);
  } else {  // NFC / NFKC / NFD / NFKD / ...: identity, loudly
    std::fprintf(stderr, "ragk tokenizer: normalizer %s not implemented (treated as identity)\n", t.c_str());
    return;
  }
  norm_.push_back(st);
}

// HF spm_precompiled semantics: darts-clone common-prefix search over the chunk's bytes (stops
// at NUL); the FIRST (shortest) hit's replacement string replaces the whole chunk.
bool Tokenizer::pc_transform(const char* p, size_t n, std::string& out) const {
  if (pc_trie_.empty()) return false;
  auto offset = [](uint32_t u) { return (u >> 10) << ((u & (1u << 9)) >> 6); };
  auto label = [](uint32_t u) { return u & ((1u << 31) | 0xFFu); };
  auto has_leaf = [](uint32_t u) { return ((u >> 8) & 1u) == 1u; };
  auto value = [](uint32_t u) { return u & ((1u << 31) - 1); };
  size_t pos = 0;
  uint32_t unit = pc_trie_[0];
  pos ^= offset(unit);
  for (size_t i = 0; i < n; ++i) {
    const unsigned char c = (unsigned char)p[i];
    if (c == 0) break;
    pos ^= c;
    if (pos >= pc_trie_.size()) return false;
    unit = pc_trie_[pos];
    if (label(unit) != c) return false;
    pos ^= offset(unit);
    if (pos >= pc_trie_.size()) return false;
    if (has_leaf(unit)) {
      const size_t v = value(pc_trie_[pos]);
      if (v >= pc_norm_.size()) return false;
      size_t e = v;
      while (e < pc_norm_.size() && pc_norm_[e] != 0) ++e;
      out.append(pc_norm_, v, e - v);
      return true;
    }
  }
  return false;
}

static bool is_gext(uint32_t c) { return in_ranges(UNI_GEXT, UNI_GEXT_N, c); }

std::string Tokenizer::normalize(const std::string& in) const {
  std::string s = in;
  for (const NormStep& st : norm_) {
    switch (st.kind) {
      case NormStep::PRECOMPILED: {
        if (pc_trie_.empty()) break;
        // walk (approximate) extended grapheme clusters: base + extending marks / ZWJ sequences,
        // CR LF, regional-indicator pairs
        std::vector<uint32_t> cps = utf8_decode(s);
        std::string out;
        size_t i = 0;
        while (i < cps.size()) {
          size_t j = i + 1;
          if (cps[i] == '\r' && j < cps.size() && cps[j] == '\n') {
            ++j;
          } else if (cps[i] >= 0x1F1E6 && cps[i] <= 0x1F1FF && j < cps.size() && cps[j] >= 0x1F1E6 &&
                     cps[j] <= 0x1F1FF) {
            ++j;
          } else {
            while (j < cps.size()) {
              if (is_gext(cps[j])) {
                ++j;
                if (cps[j - 1] == 0x200D && j < cps.size()) ++j;  // ZWJ joins the next code point
              } else {
                break;
              }
            }
          }
          const std::string g = utf8_encode(cps, i, j);
          if (!(g.size() < 6 && pc_transform(g.data(), g.size(), out))) {
            for (size_t k = i; k < j; ++k) {
              const std::string ch = utf8_encode(cps, k, k + 1);
              if (!pc_transform(ch.data(), ch.size(), out)) out += ch;
            }
          }
          i = j;
        }
        s.swap(out);
        break;
      }
      case NormStep::STRIP: {
        std::vector<uint32_t> cps = utf8_decode(s);
        size_t b = 0, e = cps.size();
        if (st.left) while (b < e && is_WS(cps[b])) ++b;
        if (st.right) while (e > b && is_WS(cps[e - 1])) --e;
        s = utf8_encode(cps, b, e);
        break;
      }
      case NormStep::REPLACE: {
        std::string out;
        size_t pos = 0;
        while (true) {
          const size_t f = s.find(st.pat, pos);
          if (f == std::string::npos) break;
          out.append(s, pos, f - pos);
          out += st.content;
          pos = f + st.pat.size();
        }
        out.append(s, pos, std::string::npos);
        s.swap(out);
        break;
      }
      case NormStep::REPLACE_RUN: {
        std::vector<uint32_t> cps = utf8_decode(s);
        std::string out;
        size_t i = 0;
        while (i < cps.size()) {
          size_t j = i;
          while (j < cps.size() && cps[j] == st.run_cp) ++j;
          if (j - i >= (size_t)st.run_min) {
            out += st.content;
            i = j;
          } else if (j > i) {
            out += utf8_encode(cps, i, j);
            i = j;
          } else {
            out += utf8_encode(cps, i, i + 1);
            ++i;
          }
        }
        s.swap(out);
        break;
      }
      case NormStep::LOWER: {
        std::vector<uint32_t> cps = utf8_decode(s);
        for (uint32_t& c : cps) c = map_lookup(UNI_LOWER, UNI_LOWER_N, c);
        s = utf8_encode(cps, 0, cps.size());
        break;
      }
      case NormStep::BERT: {
        std::vector<uint32_t> cps = utf8_decode(s), nc;
        nc.reserve(cps.size());
        for (uint32_t c : cps) {
          if (bn_clean_) {
            if (c == 0 || c == 0xFFFD || in_ranges(UNI_CTRL, UNI_CTRL_N, c)) continue;
            if (is_WS(c)) c = ' ';
          }
          if (bn_chinese_ && is_cjk(c)) {
            nc.push_back(' ');
            nc.push_back(c);
            nc.push_back(' ');
            continue;
          }
          if (bn_lower_) c = map_lookup(UNI_LOWER, UNI_LOWER_N, c);
          if (bn_strip_) {
            if (in_ranges(UNI_MN, UNI_MN_N, c)) continue;
            c = map_lookup(UNI_STRIP, UNI_STRIP_N, c);
          }
          nc.push_back(c);
        }
        s = utf8_encode(nc, 0, nc.size());
        break;
      }
    }
  }
  return s;
}

void Tokenizer::load_pre(const Json* p) {
  if (!p || p->is_null()) return;
  const std::string t = p->at("type").str;
  if (t == "Sequence") {
    for (auto& x : p->at("pretokenizers").arr) load_pre(&x);
  } else if (t == "ByteLevel") {
    byte_level_ = true;
    if (const Json* x = p->get("add_prefix_space")) add_prefix_space_ = x->truthy();
    const Json* ur = p->get("use_regex");
    if ((!ur || ur->truthy()) && pre_ == PRE_NONE) pre_ = PRE_GPT2;
  } else if (t == "Split") {
    const Json& pat = p->at("pattern");
    const std::string rx = pat.get("Regex") ? pat.at("Regex").str : pat.at("String").str;
    if (rx.find("\\p{N}{1,3}") != std::string::npos) pre_ = PRE_LLAMA3;
    else if (rx.find("?\\p{L}+| ?\\p{N}+") != std::string::npos) pre_ = PRE_GPT2;
    else throw std::runtime_error("unsupported Split pattern: " + rx);
  } else if (t == "BertPreTokenizer") {
    pre_ = PRE_BERT;
  } else if (t == "Whitespace" || t == "WhitespaceSplit") {
    pre_ = PRE_WHITESPACE;
  } else if (t == "Metaspace") {
    pre_ = PRE_METASPACE;
    if (const Json* r = p->get("replacement")) metaspace_ = r->str;
    if (const Json* ps = p->get("prepend_scheme")) meta_prepend_ = ps->str != "never";
    else if (const Json* ap = p->get("add_prefix_space")) meta_prepend_ = ap->truthy();
  } else {
    throw std::runtime_error("unsupported pre_tokenizer " + t);
  }
}

void Tokenizer::load_post(const Json* p) {
  if (!p || p->is_null()) return;
  const std::string t = p->at("type").str;
  if (t == "Sequence") {
    for (auto& x : p->at("processors").arr) load_post(&x);
  } else if (t == "TemplateProcessing") {
    has_template_ = true;
    template_single_.clear();
    const Json& sp = p->at("special_tokens");
    for (auto& item : p->at("single").arr) {
      if (const Json* s = item.get("SpecialToken")) {
        const Json& st = sp.at(s->at("id").str);
        for (auto& idv : st.at("ids").arr) template_single_.push_back((int)idv.as_int());
      } else {
        template_single_.push_back(-1);
      }
    }
  } else if (t == "BertProcessing" || t == "RobertaProcessing") {
    has_template_ = true;
    template_single_ = {(int)p->at("cls").arr.at(1).as_int(), -1, (int)p->at("sep").arr.at(1).as_int()};
  }
}

void Tokenizer::load_decoder(const Json* d) {
  if (!d || d->is_null()) return;
  const std::string t = d->at("type").str;
  if (t == "Sequence") {
    for (auto& x : d->at("decoders").arr) load_decoder(&x);
  } else if (t == "ByteLevel") {
    dec_ = DEC_BYTELEVEL;
  } else if (t == "WordPiece") {
    dec_ = DEC_WORDPIECE;
    if (const Json* x = d->get("prefix")) wp_prefix_ = x->str;
    if (const Json* x = d->get("cleanup")) wp_cleanup_ = x->truthy();
  } else if (t == "Metaspace") {
    dec_ = DEC_METASPACE;
  }
}

int Tokenizer::token_to_id(const std::string& t) const {
  auto it = vocab_.find(t);
  return it == vocab_.end() ? -1 : it->second;
}

void Tokenizer::bpe_word(const std::string& word, std::vector<int>& out, WordCache* local) const {
  if (local) {  // encode_batch worker: private cache, no locking
    auto c = local->find(word);
    if (c != local->end()) {
      out.insert(out.end(), c->second.begin(), c->second.end());
      return;
    }
  } else {  // shared word cache: encode() runs without the GIL from several server threads
    std::shared_lock<std::shared_mutex> rd(cache_mu_);
    auto c = cache_.find(word);
    if (c != cache_.end()) {
      out.insert(out.end(), c->second.begin(), c->second.end());
      return;
    }
  }
  std::vector<int> ids;
  auto whole = vocab_.find(word);
  if (ignore_merges_ && whole != vocab_.end()) {
    ids.push_back(whole->second);
  } else {
    const std::vector<uint32_t> cps = utf8_decode(word);
    for (uint32_t cp : cps) {
      auto it = vocab_.find(cp_utf8(cp));
      if (it != vocab_.end()) {
        ids.push_back(it->second);
      } else if (byte_fallback_) {
        const std::string u = cp_utf8(cp);
        for (unsigned char b : u) {
          char buf[8];
          snprintf(buf, sizeof(buf), "<0x%02X>", b);
          auto f = vocab_.find(buf);
          if (f != vocab_.end()) ids.push_back(f->second);
        }
      }
    }
    while (ids.size() > 1) {
      int best = std::numeric_limits<int>::max(), bi = -1, merged = -1;
      for (size_t i = 0; i + 1 < ids.size(); ++i) {
        const uint64_t key = ((uint64_t)(uint32_t)ids[i] << 32) | (uint32_t)ids[i + 1];
        auto it = merges_.find(key);
        if (it != merges_.end() && it->second.first < best) {
          best = it->second.first;
          bi = (int)i;
          merged = it->second.second;
        }
      }
      if (bi < 0) break;
      ids[bi] = merged;
      ids.erase(ids.begin() + bi + 1);
    }
  }
  if (local) {
    if (local->size() < 200000) local->emplace(word, ids);
  } else {
    std::unique_lock<std::shared_mutex> wr(cache_mu_);
    if (cache_.size() < 200000) cache_.emplace(word, ids);
  }
  out.insert(out.end(), ids.begin(), ids.end());
}

namespace {

// Process-wide worker pool for encode_batch. Workers live for the process, so their per-thread
// BPE word caches (keyed by tokenizer uid) stay warm across calls.
class EncodePool {
 public:
  static EncodePool& get() {
    static EncodePool p;
    return p;
  }
  int size() const { return (int)threads_.size(); }
  // run fn(worker_index) on `n` workers and wait. One job at a time: concurrent callers (server
  // threads tokenizing long prompts while the batcher encodes) queue on call_mu_ -- the job slot
  // (job_ / want_ / started_ / done_) is shared by all workers.
  void run(int n, const std::function<void(int)>& fn) {
    std::lock_guard<std::mutex> one(call_mu_);
    std::unique_lock<std::mutex> lk(mu_);
    job_ = &fn;
    want_ = std::min(n, size());
    started_ = 0;
    done_ = 0;
    ++gen_;
    cv_.notify_all();
    done_cv_.wait(lk, [&] { return done_ == want_; });
    job_ = nullptr;
  }

 private:
  EncodePool() {
    const int n = std::max(1, std::min(16, (int)std::thread::hardware_concurrency()));
    for (int i = 0; i < n; ++i) threads_.emplace_back([this] { loop(); });
  }
  ~EncodePool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      cv_.notify_all();
    }
    for (auto& t : threads_) t.join();
  }
  void loop() {
    unsigned long long seen = 0;
    std::unique_lock<std::mutex> lk(mu_);
    while (true) {
      cv_.wait(lk, [&] { return stop_ || (gen_ != seen && started_ < want_); });
      if (stop_) return;
      if (started_ >= want_) {
        seen = gen_;
        continue;
      }
      const int idx = started_++;
      seen = gen_;
      const std::function<void(int)>* fn = job_;
      lk.unlock();
      (*fn)(idx);
      lk.lock();
      if (++done_ == want_) done_cv_.notify_all();
    }
  }
  std::vector<std::thread> threads_;
  std::mutex call_mu_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* job_ = nullptr;
  int want_ = 0, started_ = 0, done_ = 0;
  unsigned long long gen_ = 0;
  bool stop_ = false;
};

}  // namespace

std::vector<std::vector<int>> Tokenizer::encode_batch(const std::vector<std::string>& texts, bool add_special,
                                                      int threads, int max_tokens) const {
  std::vector<std::vector<int>> out(texts.size());
  const int n = (int)texts.size();
  const size_t budget = max_tokens < 0 ? SIZE_MAX : (size_t)max_tokens;
  EncodePool& pool = EncodePool::get();
  const int nt = std::max(1, std::min({threads, n, pool.size()}));
  if (nt == 1) {
    for (int i = 0; i < n; ++i) out[i] = encode_impl(texts[i], add_special, nullptr, budget);
    return out;
  }
  std::atomic<int> next{0};
  std::exception_ptr err = nullptr;
  std::mutex err_mu;
  const unsigned long long uid = uid_;
  pool.run(nt, [&](int) {
    thread_local std::unordered_map<unsigned long long, WordCache> caches;
    WordCache& local = caches[uid];
    try {
      for (int i = next++; i < n; i = next++) out[i] = encode_impl(texts[i], add_special, &local, budget);
    } catch (...) {
      std::lock_guard<std::mutex> g(err_mu);
      if (!err) err = std::current_exception();
    }
  });
  if (err) std::rethrow_exception(err);
  return out;
}

void Tokenizer::wordpiece_word(const std::vector<uint32_t>& cps, std::vector<int>& out) const {
  const int unk = token_to_id(unk_token_);
  if ((int)cps.size() > max_chars_per_word_) {
    out.push_back(unk);
    return;
  }
  std::vector<int> pieces;
  size_t start = 0;
  while (start < cps.size()) {
    size_t end = cps.size();
    int cur = -1;
    while (start < end) {
      std::string sub = utf8_encode(cps, start, end);
      if (start > 0) sub = wp_prefix_ + sub;
      auto it = vocab_.find(sub);
      if (it != vocab_.end()) {
        cur = it->second;
        break;
      }
      --end;
    }
    if (cur < 0) {
      out.push_back(unk);
      return;
    }
    pieces.push_back(cur);
    start = end;
  }
  out.insert(out.end(), pieces.begin(), pieces.end());
}

void Tokenizer::unigram_word(const std::string& word, std::vector<int>& out) const {
  const std::vector<uint32_t> cps = utf8_decode(word);
  const size_t n = cps.size();
  const double NEG = -std::numeric_limits<double>::infinity();
  std::vector<double> best(n + 1, NEG);
  std::vector<int> from(n + 1, -1), tok(n + 1, -1);
  best[0] = 0;
  const double unk_score = min_score_ - 10.0;
  for (size_t i = 0; i < n; ++i) {
    if (best[i] == NEG) continue;
    bool single = false;
    std::string sub;
    for (size_t e = i + 1; e <= n && e - i <= 64; ++e) {
      append_utf8(sub, cps[e - 1]);
      auto it = vocab_.find(sub);
      if (it != vocab_.end() && it->second < (int)scores_.size()) {
        const double s = best[i] + scores_[it->second];
        if (s > best[e]) {
          best[e] = s;
          from[e] = (int)i;
          tok[e] = it->second;
        }
        if (e == i + 1) single = true;
      }
    }
    if (!single && best[i] + unk_score > best[i + 1]) {
      best[i + 1] = best[i] + unk_score;
      from[i + 1] = (int)i;
      tok[i + 1] = unk_id_;
    }
  }
  std::vector<int> rev;
  for (int e = (int)n; e > 0; e = from[e]) rev.push_back(tok[e]);
  std::reverse(rev.begin(), rev.end());
  int prev = -2;
  for (int t : rev) {  // fuse consecutive unknowns
    if (t == unk_id_ && prev == unk_id_) continue;
    out.push_back(t);
    prev = t;
  }
}

void Tokenizer::encode_segment(const std::string& seg, std::vector<int>& out, WordCache* local, size_t budget) const {
  // Truncated encode of a long text with a per-character normalizer and whitespace-delimited words
  // (BERT WordPiece: MiniLM / bge-large ingest of 1000-word chunks truncated to 256 / 512 tokens):
  // normalise and split only as much text as the budget needs, in slices cut at ASCII whitespace (a
  // word boundary before and after normalisation), instead of the whole chunk.
  if (budget != SIZE_MAX && slice_safe_ && seg.size() > 2048) {
    size_t pos = 0;
    while (pos < seg.size() && out.size() < budget) {
      size_t end = std::min(seg.size(), pos + std::max<size_t>(1024, (budget - out.size()) * 8));
      while (end < seg.size() && seg[end] != ' ' && seg[end] != '\t' && seg[end] != '\n' && seg[end] != '\r') ++end;
      encode_words(seg.substr(pos, end - pos), out, local, budget);
      pos = end;
    }
    return;
  }
  encode_words(seg, out, local, budget);
}

void Tokenizer::encode_words(const std::string& seg, std::vector<int>& out, WordCache* local, size_t budget) const {
  std::vector<uint32_t> cps = utf8_decode(norm_.empty() ? seg : normalize(seg));
  std::vector<std::pair<size_t, size_t>> words;
  const size_t n = cps.size();
  if (pre_ == PRE_GPT2 || pre_ == PRE_LLAMA3) {
    size_t i = 0;
    while (i < n) {
      size_t k = pre_ == PRE_GPT2 ? match_gpt2(cps, i) : match_llama3(cps, i);
      if (k == 0) k = 1;
      words.push_back({i, i + k});
      i += k;
    }
  } else if (pre_ == PRE_BERT || pre_ == PRE_WHITESPACE) {
    size_t i = 0;
    while (i < n) {
      if (is_WS(cps[i])) { ++i; continue; }
      if (pre_ == PRE_BERT && is_bert_punct(cps[i])) {
        words.push_back({i, i + 1});
        ++i;
        continue;
      }
      size_t j = i;
      while (j < n && !is_WS(cps[j]) && !(pre_ == PRE_BERT && is_bert_punct(cps[j]))) ++j;
      words.push_back({i, j});
      i = j;
    }
  } else if (pre_ == PRE_METASPACE) {
    const uint32_t meta = utf8_decode(metaspace_)[0];
    std::vector<uint32_t> m;
    if (meta_prepend_ && (n == 0 || (cps[0] != ' ' && cps[0] != meta))) m.push_back(meta);
    for (uint32_t c : cps) m.push_back(c == ' ' ? meta : c);
    cps.swap(m);
    size_t i = 0;
    const size_t nn = cps.size();
    while (i < nn) {
      size_t j = i + 1;
      while (j < nn && cps[j] != meta) ++j;
      words.push_back({i, j});
      i = j;
    }
  } else if (n) {
    words.push_back({0, n});
  }
  for (auto& w : words) {
    if (out.size() >= budget) break;  // truncated encode: later words cannot change this prefix
    std::string piece = utf8_encode(cps, w.first, w.second);
    if (model_ == BPE) {
      if (byte_level_) {
        std::string mapped;
        for (unsigned char b : piece) mapped += byte_to_uni_[b];
        piece.swap(mapped);
      }
      bpe_word(piece, out, local);
    } else {
      // WordPiece / Unigram: memoised per word in the batch worker's private cache (Zipfian text
      // repeats words; no lock on this path)
      if (local) {
        auto c = local->find(piece);
        if (c != local->end()) {
          out.insert(out.end(), c->second.begin(), c->second.end());
          continue;
        }
      }
      std::vector<int> ids;
      if (model_ == WORDPIECE) wordpiece_word(std::vector<uint32_t>(cps.begin() + w.first, cps.begin() + w.second), ids);
      else unigram_word(piece, ids);
      out.insert(out.end(), ids.begin(), ids.end());
      if (local && local->size() < 200000) local->emplace(std::move(piece), std::move(ids));
    }
  }
}

std::vector<int> Tokenizer::encode(const std::string& text, bool add_special_tokens, int max_tokens) const {
  return encode_impl(text, add_special_tokens, nullptr, max_tokens < 0 ? SIZE_MAX : (size_t)max_tokens);
}

std::vector<int> Tokenizer::encode_impl(const std::string& text, bool add_special_tokens, WordCache* local,
                                        size_t budget) const {
  std::vector<int> body;
  size_t seg_start = 0, i = 0;
  const size_t n = text.size();
  while (i < n && body.size() < budget) {
    if (!added_first_bytes_.empty() && added_first_bytes_.count((unsigned char)text[i])) {
      bool hit = false;
      for (auto& a : added_) {
        if (!a.content.empty() && text.compare(i, a.content.size(), a.content) == 0) {
          if (i > seg_start) encode_segment(text.substr(seg_start, i - seg_start), body, local, budget);
          body.push_back(a.id);
          i += a.content.size();
          seg_start = i;
          hit = true;
          break;
        }
      }
      if (hit) continue;
    }
    ++i;
  }
  if (seg_start < n && body.size() < budget) encode_segment(text.substr(seg_start), body, local, budget);
  if (!add_special_tokens || !has_template_) return body;
  std::vector<int> out;
  for (int t : template_single_) {
    if (t < 0) out.insert(out.end(), body.begin(), body.end());
    else out.push_back(t);
  }
  return out;
}

std::string Tokenizer::decode(const std::vector<int>& ids, bool skip_special_tokens) const {
  std::vector<std::string> toks;
  for (int id : ids) {
    if (id < 0 || id >= (int)id_to_tok_.size()) continue;
    if (skip_special_tokens && special_ids_.count(id)) continue;
    toks.push_back(id_to_tok_[id]);
  }
  if (dec_ == DEC_BYTELEVEL) {
    std::string bytes;
    for (auto& t : toks)
      for (uint32_t cp : utf8_decode(t)) {
        auto it = uni_to_byte_.find(cp);
        if (it != uni_to_byte_.end()) bytes += (char)it->second;
        else append_utf8(bytes, cp);
      }
    return utf8_encode(utf8_decode(bytes), 0, utf8_decode(bytes).size());  // lossy UTF-8 repair
  }
  if (dec_ == DEC_WORDPIECE) {
    std::string s;
    for (size_t i = 0; i < toks.size(); ++i) {
      const std::string& t = toks[i];
      if (i == 0) s += t;
      else if (t.compare(0, wp_prefix_.size(), wp_prefix_) == 0) s += t.substr(wp_prefix_.size());
      else s += " " + t;
    }
    if (wp_cleanup_) {
      static const char* pairs[][2] = {{" .", "."}, {" ?", "?"}, {" !", "!"}, {" ,", ","}, {" ' ", "'"},
                                       {" n't", "n't"}, {" 'm", "'m"}, {" do not", " don't"}, {" 's", "'s"},
                                       {" 've", "'ve"}, {" 're", "'re"}};
      for (auto& p : pairs) {
        std::string out;
        const std::string a = p[0], b = p[1];
        size_t pos = 0, f;
        while ((f = s.find(a, pos)) != std::string::npos) {
          out += s.substr(pos, f - pos) + b;
          pos = f + a.size();
        }
        out += s.substr(pos);
        s.swap(out);
      }
    }
    return s;
  }
  std::string s;
  for (auto& t : toks) s += t;
  if (dec_ == DEC_METASPACE) {
    std::string out;
    size_t pos = 0, f;
    while ((f = s.find(metaspace_, pos)) != std::string::npos) {
      out += s.substr(pos, f - pos) + " ";
      pos = f + metaspace_.size();
    }
    out += s.substr(pos);
    if (!out.empty() && out[0] == ' ') out.erase(0, 1);
    return out;
  }
  return s;
}

}  // namespace ragk_rt
