// Minimal JSON reader for the deploy manifest (objects, arrays, strings,
// numbers, true/false/null).  Host only.
#pragma once
#include <cstdlib>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace minijson {

struct Value {
  enum Kind { NUL, BOOL, NUM, STR, ARR, OBJ } kind = NUL;
  double n = 0;
  bool b = false;
  std::string s;
  std::vector<Value> a;
  std::map<std::string, Value> o;

  const Value& operator[](const std::string& k) const {
    if (kind != OBJ) throw std::runtime_error("not an object at key " + k);
    auto it = o.find(k);
    if (it == o.end()) throw std::runtime_error("missing key " + k);
    return it->second;
  }
  bool has(const std::string& k) const { return kind == OBJ && o.count(k) != 0; }
  double num() const {
    if (kind != NUM) throw std::runtime_error("not a number");
    return n;
  }
  bool boolean() const {
    if (kind != BOOL) throw std::runtime_error("not a boolean");
    return b;
  }
  const std::string& str() const {
    if (kind != STR) throw std::runtime_error("not a string");
    return s;
  }
  const std::vector<Value>& arr() const {
    if (kind != ARR) throw std::runtime_error("not an array");
    return a;
  }
};

namespace detail {
struct P {
  const std::string& t;
  size_t i = 0;
  void ws() {
    while (i < t.size() && (t[i] == ' ' || t[i] == '\n' || t[i] == '\r' || t[i] == '\t')) ++i;
  }
  char peek() {
    ws();
    if (i >= t.size()) throw std::runtime_error("unexpected end");
    return t[i];
  }
  void expect(char c) {
    if (peek() != c) throw std::runtime_error(std::string("expected ") + c);
    ++i;
  }
  std::string str() {
    expect('"');
    std::string out;
    while (i < t.size() && t[i] != '"') {
      if (t[i] == '\\') {
        ++i;
        const char c = t[i];
        if (c == 'n') out += '\n';
        else if (c == 't') out += '\t';
        else if (c == 'u') {
          out += '?';
          i += 4;
        } else out += c;
        ++i;
      } else {
        out += t[i++];
      }
    }
    if (i >= t.size()) throw std::runtime_error("unterminated string");
    ++i;
    return out;
  }
  void val(Value& v) {
    const char c = peek();
    if (c == '{') {
      v.kind = Value::OBJ;
      ++i;
      if (peek() == '}') {
        ++i;
        return;
      }
      for (;;) {
        std::string k = str();
        expect(':');
        val(v.o[k]);
        if (peek() == ',') {
          ++i;
          continue;
        }
        expect('}');
        return;
      }
    } else if (c == '[') {
      v.kind = Value::ARR;
      ++i;
      if (peek() == ']') {
        ++i;
        return;
      }
      for (;;) {
        v.a.emplace_back();
        val(v.a.back());
        if (peek() == ',') {
          ++i;
          continue;
        }
        expect(']');
        return;
      }
    } else if (c == '"') {
      v.kind = Value::STR;
      v.s = str();
    } else if (t.compare(i, 4, "true") == 0) {
      v.kind = Value::BOOL;
      v.b = true;
      i += 4;
    } else if (t.compare(i, 5, "false") == 0) {
      v.kind = Value::BOOL;
      i += 5;
    } else if (t.compare(i, 4, "null") == 0) {
      i += 4;
    } else {
      char* end = nullptr;
      v.kind = Value::NUM;
      v.n = std::strtod(t.c_str() + i, &end);
      if (end == t.c_str() + i) throw std::runtime_error("bad token");
      i = end - t.c_str();
    }
  }
};
}  // namespace detail

inline bool parse(const std::string& text, Value& out, std::string& err) {
  try {
    detail::P p{text};
    p.val(out);
    return true;
  } catch (const std::exception& e) {
    err = e.what();
    return false;
  }
}

}  // namespace minijson
