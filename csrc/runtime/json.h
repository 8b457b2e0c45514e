// Minimal DOM JSON parser for the host runtime (tokenizer.json, safetensors headers,
// *.index.json). UTF-8 in/out, \uXXXX escapes incl. surrogate pairs, int64-exact integers.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace ragk_rt {

struct Json {
  enum Type { NUL, BOOL, NUM, STR, ARR, OBJ } type = NUL;
  bool b = false;
  double num = 0.0;
  int64_t i64 = 0;
  bool is_int = false;
  std::string str;
  std::vector<Json> arr;
  std::vector<std::pair<std::string, Json>> obj;  // insertion order preserved

  bool is_null() const { return type == NUL; }
  const Json* get(const std::string& k) const {
    if (type != OBJ) return nullptr;
    for (auto& kv : obj)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  const Json& at(const std::string& k) const {
    const Json* j = get(k);
    if (!j) throw std::runtime_error("json: missing key " + k);
    return *j;
  }
  int64_t as_int() const { return is_int ? i64 : (int64_t)num; }
  double as_num() const { return is_int ? (double)i64 : num; }
  bool truthy() const { return type == BOOL ? b : (type == NUM ? as_num() != 0 : type != NUL); }
};

inline void append_utf8(std::string& out, uint32_t cp) {
  if (cp < 0x80) {
    out += (char)cp;
  } else if (cp < 0x800) {
    out += (char)(0xC0 | (cp >> 6));
    out += (char)(0x80 | (cp & 0x3F));
  } else if (cp < 0x10000) {
    out += (char)(0xE0 | (cp >> 12));
    out += (char)(0x80 | ((cp >> 6) & 0x3F));
    out += (char)(0x80 | (cp & 0x3F));
  } else {
    out += (char)(0xF0 | (cp >> 18));
    out += (char)(0x80 | ((cp >> 12) & 0x3F));
    out += (char)(0x80 | ((cp >> 6) & 0x3F));
    out += (char)(0x80 | (cp & 0x3F));
  }
}

class JsonParser {
 public:
  JsonParser(const char* p, size_t n) : s_(p), e_(p + n) {}
  Json parse() {
    Json v = value();
    ws();
    if (s_ != e_) fail("trailing characters");
    return v;
  }

 private:
  const char* s_;
  const char* e_;

  [[noreturn]] void fail(const char* m) { throw std::runtime_error(std::string("json parse error: ") + m); }
  void ws() {
    while (s_ < e_ && (*s_ == ' ' || *s_ == '\n' || *s_ == '\r' || *s_ == '\t')) ++s_;
  }
  Json value() {
    ws();
    if (s_ >= e_) fail("unexpected end");
    char c = *s_;
    if (c == '{') return object();
    if (c == '[') return array();
    if (c == '"') {
      Json j;
      j.type = Json::STR;
      j.str = string();
      return j;
    }
    if (c == 't' || c == 'f') {
      Json j;
      j.type = Json::BOOL;
      if (e_ - s_ >= 4 && std::string(s_, 4) == "true") {
        j.b = true;
        s_ += 4;
      } else if (e_ - s_ >= 5 && std::string(s_, 5) == "false") {
        s_ += 5;
      } else {
        fail("bad literal");
      }
      return j;
    }
    if (c == 'n') {
      if (e_ - s_ >= 4 && std::string(s_, 4) == "null") {
        s_ += 4;
        return Json();
      }
      fail("bad literal");
    }
    return number();
  }
  Json number() {
    const char* st = s_;
    bool isint = true;
    if (*s_ == '-') ++s_;
    while (s_ < e_ && ((*s_ >= '0' && *s_ <= '9') || *s_ == '.' || *s_ == 'e' || *s_ == 'E' || *s_ == '+' ||
                       *s_ == '-')) {
      if (*s_ == '.' || *s_ == 'e' || *s_ == 'E') isint = false;
      ++s_;
    }
    std::string t(st, s_);
    if (t.empty()) fail("bad number");
    Json j;
    j.type = Json::NUM;
    if (isint) {
      j.is_int = true;
      j.i64 = std::stoll(t);
      j.num = (double)j.i64;
    } else {
      j.num = std::stod(t);
    }
    return j;
  }
  uint32_t hex4() {
    if (e_ - s_ < 4) fail("short \\u escape");
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) {
      char c = *s_++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad hex");
    }
    return v;
  }
  std::string string() {
    ++s_;  // opening quote
    std::string out;
    while (true) {
      if (s_ >= e_) fail("unterminated string");
      char c = *s_++;
      if (c == '"') break;
      if (c != '\\') {
        out += c;
        continue;
      }
      if (s_ >= e_) fail("bad escape");
      char e = *s_++;
      switch (e) {
        case '"': out += '"'; break;
        case '\\': out += '\\'; break;
        case '/': out += '/'; break;
        case 'b': out += '\b'; break;
        case 'f': out += '\f'; break;
        case 'n': out += '\n'; break;
        case 'r': out += '\r'; break;
        case 't': out += '\t'; break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp <= 0xDBFF && e_ - s_ >= 6 && s_[0] == '\\' && s_[1] == 'u') {
            s_ += 2;
            uint32_t lo = hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          append_utf8(out, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
    return out;
  }
  Json array() {
    ++s_;
    Json j;
    j.type = Json::ARR;
    ws();
    if (s_ < e_ && *s_ == ']') {
      ++s_;
      return j;
    }
    while (true) {
      j.arr.push_back(value());
      ws();
      if (s_ >= e_) fail("unterminated array");
      if (*s_ == ',') { ++s_; continue; }
      if (*s_ == ']') { ++s_; break; }
      fail("expected , or ]");
    }
    return j;
  }
  Json object() {
    ++s_;
    Json j;
    j.type = Json::OBJ;
    ws();
    if (s_ < e_ && *s_ == '}') {
      ++s_;
      return j;
    }
    while (true) {
      ws();
      if (s_ >= e_ || *s_ != '"') fail("expected key");
      std::string k = string();
      ws();
      if (s_ >= e_ || *s_ != ':') fail("expected :");
      ++s_;
      j.obj.emplace_back(std::move(k), value());
      ws();
      if (s_ >= e_) fail("unterminated object");
      if (*s_ == ',') { ++s_; continue; }
      if (*s_ == '}') { ++s_; break; }
      fail("expected , or }");
    }
    return j;
  }
};

inline Json parse_json(const std::string& s) { return JsonParser(s.data(), s.size()).parse(); }

}  // namespace ragk_rt
