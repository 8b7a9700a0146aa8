// Minimal JSON reader for the sg_app_create descriptor (host side of the C ABI; the oracle
// oracle/siddhi_oracle.cpp reads the same descriptors with it).
#pragma once
#include <cstdint>
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace sgjson {

struct J {
  enum K { NUL, BOOL, NUM, STR, ARR, OBJ } k = NUL;
  bool b = false;
  double n = 0;
  bool is_int = false;
  int64_t i = 0;
  std::string s;
  std::vector<J> a;
  std::vector<std::pair<std::string, J>> o;

  bool null() const { return k == NUL; }
  const J& operator[](const std::string& key) const {
    static J nul;
    for (auto& kv : o) if (kv.first == key) return kv.second;
    return nul;
  }
  bool has(const std::string& key) const {
    for (auto& kv : o) if (kv.first == key) return true;
    return false;
  }
  const J& operator[](size_t idx) const { return a.at(idx); }
  size_t size() const { return k == ARR ? a.size() : o.size(); }
  int64_t as_int() const { return is_int ? i : (int64_t)n; }
};

struct Reader {
  const char* p;
  const char* end;
  explicit Reader(const std::string& s) : p(s.data()), end(s.data() + s.size()) {}
  void ws() { while (p < end && (*p == ' ' || *p == '\n' || *p == '\t' || *p == '\r')) ++p; }
  [[noreturn]] void fail(const char* m) { throw std::runtime_error(std::string("json: ") + m); }
  J parse() {
    ws();
    J j;
    if (p >= end) fail("eof");
    char c = *p;
    if (c == '{') {
      j.k = J::OBJ; ++p; ws();
      if (*p == '}') { ++p; return j; }
      while (true) {
        ws(); J key = parse(); ws();
        if (*p != ':') fail("expected :"); ++p;
        J v = parse();
        j.o.emplace_back(key.s, std::move(v));
        ws();
        if (*p == ',') { ++p; continue; }
        if (*p == '}') { ++p; break; }
        fail("expected , or }");
      }
    } else if (c == '[') {
      j.k = J::ARR; ++p; ws();
      if (*p == ']') { ++p; return j; }
      while (true) {
        j.a.push_back(parse()); ws();
        if (*p == ',') { ++p; continue; }
        if (*p == ']') { ++p; break; }
        fail("expected , or ]");
      }
    } else if (c == '"') {
      j.k = J::STR; ++p;
      while (p < end && *p != '"') {
        if (*p == '\\') {
          ++p;
          char e = *p++;
          switch (e) {
            case 'n': j.s += '\n'; break;
            case 't': j.s += '\t'; break;
            case 'r': j.s += '\r'; break;
            case 'b': j.s += '\b'; break;
            case 'f': j.s += '\f'; break;
            case 'u': {
              unsigned cp = std::strtoul(std::string(p, p + 4).c_str(), nullptr, 16); p += 4;
              if (cp < 0x80) j.s += (char)cp;
              else if (cp < 0x800) { j.s += (char)(0xC0 | (cp >> 6)); j.s += (char)(0x80 | (cp & 0x3F)); }
              else { j.s += (char)(0xE0 | (cp >> 12)); j.s += (char)(0x80 | ((cp >> 6) & 0x3F)); j.s += (char)(0x80 | (cp & 0x3F)); }
              break;
            }
            default: j.s += e;
          }
        } else {
          j.s += *p++;
        }
      }
      ++p;
    } else if (c == 't' && end - p >= 4 && std::string(p, p + 4) == "true") { j.k = J::BOOL; j.b = true; p += 4; }
    else if (c == 'f' && end - p >= 5 && std::string(p, p + 5) == "false") { j.k = J::BOOL; j.b = false; p += 5; }
    else if (c == 'n' && end - p >= 4 && std::string(p, p + 4) == "null") { j.k = J::NUL; p += 4; }
    else {
      const char* st = p;
      bool isint = true;
      if (*p == '-' || *p == '+') ++p;
      while (p < end && ((*p >= '0' && *p <= '9') || *p == '.' || *p == 'e' || *p == 'E' || *p == '-' || *p == '+')) {
        if (*p == '.' || *p == 'e' || *p == 'E') isint = false;
        ++p;
      }
      std::string num(st, p);
      if (num.empty()) fail("bad token");
      j.k = J::NUM;
      j.n = std::strtod(num.c_str(), nullptr);
      if (isint) { j.is_int = true; j.i = std::strtoll(num.c_str(), nullptr, 10); }
      // Infinity / NaN spellings from Python json
    }
    return j;
  }
};

inline J parse(const std::string& s) {
  std::string t = s;
  Reader r(t);
  return r.parse();
}

}  // namespace sgjson
