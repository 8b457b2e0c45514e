// Native tokenizers reading HF tokenizer.json (replaces the Rust `tokenizers` crate the
// reference uses through AutoTokenizer / sentence-transformers).
//   * byte-level BPE  (Llama-3 Split regex + ByteLevel, GPT-2 ByteLevel regex), ignore_merges
//   * WordPiece       (BertNormalizer + BertPreTokenizer, greedy longest-match-first)
//   * Unigram         (Metaspace pre-tokenizer, Viterbi) with the SentencePiece
//                      Precompiled (charsmap double-array trie) normalizer of XLM-R / bge-m3
// Normalizers run as an ordered pipeline: Precompiled, Strip, Replace (literal / "c{n,}" runs),
// Lowercase, BertNormalizer; NFC/NFKC/NFD/NFKD are not implemented (identity + a warning).
// Added/special tokens are split out before normalisation; TemplateProcessing / Bert /
// Roberta post-processors; ByteLevel / WordPiece / Metaspace decoders.
#pragma once
#include <cstdint>
#include <shared_mutex>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "json.h"

namespace ragk_rt {

class Tokenizer {
 public:
  explicit Tokenizer(const std::string& path);
  // max_tokens >= 0: stop once the body holds max_tokens tokens (every model here tokenizes word by
  // word, so the result is a prefix of the full encoding: exact under right truncation to max_tokens)
  std::vector<int> encode(const std::string& text, bool add_special_tokens, int max_tokens = -1) const;  // thread-safe
  // many texts on `threads` worker threads (the per-word BPE cache is shared under a shared_mutex)
  std::vector<std::vector<int>> encode_batch(const std::vector<std::string>& texts, bool add_special_tokens,
                                             int threads, int max_tokens = -1) const;
  std::string decode(const std::vector<int>& ids, bool skip_special_tokens) const;
  int vocab_size() const { return (int)id_to_tok_.size(); }
  int token_to_id(const std::string& t) const;
  bool is_special(int id) const { return special_ids_.count(id) != 0; }
  std::string model_type() const { return model_name_; }

 private:
  enum Model { BPE, WORDPIECE, UNIGRAM } model_;
  std::string model_name_;
  std::vector<std::string> id_to_tok_;
  std::unordered_map<std::string, int> vocab_;
  // BPE
  std::unordered_map<uint64_t, std::pair<int, int>> merges_;  // (a<<32|b) -> (rank, merged id)
  bool ignore_merges_ = false;
  bool byte_fallback_ = false;
  // WordPiece
  std::string unk_token_ = "[UNK]";
  std::string wp_prefix_ = "##";
  int max_chars_per_word_ = 100;
  // Unigram
  std::vector<double> scores_;
  int unk_id_ = 0;
  double min_score_ = 0.0;
  // normalizer pipeline
  struct NormStep {
    enum Kind { PRECOMPILED, STRIP, REPLACE, REPLACE_RUN, LOWER, BERT } kind;
    bool left = false, right = false;  // STRIP
    std::string pat, content;          // REPLACE (literal); REPLACE_RUN: content
    uint32_t run_cp = 0;               // REPLACE_RUN: runs of >= run_min run_cp
    int run_min = 2;
  };
  std::vector<NormStep> norm_;
  bool bn_clean_ = true, bn_chinese_ = true, bn_lower_ = false, bn_strip_ = false;
  std::vector<uint32_t> pc_trie_;  // Precompiled: darts-clone double array units
  std::string pc_norm_;            // Precompiled: NUL-separated replacement strings
  // pre-tokenizer
  enum Pre { PRE_NONE, PRE_GPT2, PRE_LLAMA3, PRE_BERT, PRE_WHITESPACE, PRE_METASPACE } pre_ = PRE_NONE;
  bool byte_level_ = false;
  bool add_prefix_space_ = false;
  std::string metaspace_ = "\xE2\x96\x81";  // U+2581
  bool meta_prepend_ = true;
  // added tokens
  struct Added { int id; std::string content; bool special; };
  std::vector<Added> added_;
  std::unordered_set<int> special_ids_;
  std::unordered_set<unsigned char> added_first_bytes_;
  // post-processor: sequence of ids (-1 = the input sequence)
  std::vector<int> template_single_;
  bool has_template_ = false;
  // decoder
  enum Dec { DEC_NONE, DEC_BYTELEVEL, DEC_WORDPIECE, DEC_METASPACE } dec_ = DEC_NONE;
  bool wp_cleanup_ = true;
  // byte-level maps
  std::string byte_to_uni_[256];
  std::unordered_map<uint32_t, unsigned char> uni_to_byte_;
  mutable std::unordered_map<std::string, std::vector<int>> cache_;
  mutable std::shared_mutex cache_mu_;
  unsigned long long uid_ = 0;  // keys the encode_batch workers' thread-local word caches

  void load_model(const Json& m);
  void load_normalizer(const Json* n);
  void load_pre(const Json* p);
  void load_post(const Json* p);
  void load_decoder(const Json* d);
  using WordCache = std::unordered_map<std::string, std::vector<int>>;
  // local != null: a caller-owned (per-thread) word cache, used without locking
  std::vector<int> encode_impl(const std::string& text, bool add_special_tokens, WordCache* local,
                               size_t budget = SIZE_MAX) const;
  void encode_segment(const std::string& seg, std::vector<int>& out, WordCache* local,
                      size_t budget = SIZE_MAX) const;
  void encode_words(const std::string& seg, std::vector<int>& out, WordCache* local, size_t budget) const;
  bool slice_safe_ = false;  // normaliser per character + whitespace pre-tokenizer: slicing at spaces is exact
  std::string normalize(const std::string& s) const;
  bool pc_transform(const char* p, size_t n, std::string& out) const;
  void bpe_word(const std::string& word, std::vector<int>& out, WordCache* local) const;
  void wordpiece_word(const std::vector<uint32_t>& cps, std::vector<int>& out) const;
  void unigram_word(const std::string& word, std::vector<int>& out) const;
};

// helpers shared with the tests
std::vector<uint32_t> utf8_decode(const std::string& s);
std::string utf8_encode(const std::vector<uint32_t>& cps, size_t b, size_t e);

}  // namespace ragk_rt
