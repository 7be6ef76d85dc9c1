// json.cpp — parser and writer for rt2::Json (see json.h).
#include "json.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

namespace rt2 {

class JsonParser {
 public:
  JsonParser(const std::string& t) : s_(t.data()), n_(t.size()) {}

  bool Run(Json& out, std::string& err) {
    SkipWs();
    if (!Value(out, 0)) {
      err = Where() + err_;
      return false;
    }
    SkipWs();
    if (i_ != n_) {
      err = Where() + "trailing characters after the JSON document";
      return false;
    }
    return true;
  }

 private:
  const char* s_;
  size_t n_;
  size_t i_ = 0;
  std::string err_;

  std::string Where() const {
    size_t line = 1, col = 1;
    for (size_t k = 0; k < i_ && k < n_; k++) {
      if (s_[k] == '\n') {
        line++;
        col = 1;
      } else {
        col++;
      }
    }
    return "line " + std::to_string(line) + " col " + std::to_string(col) + ": ";
  }
  bool Fail(const char* m) {
    if (err_.empty()) err_ = m;
    return false;
  }
  void SkipWs() {
    while (i_ < n_ && (s_[i_] == ' ' || s_[i_] == '\t' || s_[i_] == '\n' || s_[i_] == '\r')) i_++;
  }
  bool Lit(const char* w) {
    size_t l = strlen(w);
    if (i_ + l <= n_ && memcmp(s_ + i_, w, l) == 0) {
      i_ += l;
      return true;
    }
    return false;
  }
  bool String(std::string& out) {
    if (i_ >= n_ || s_[i_] != '"') return Fail("expected '\"'");
    i_++;
    while (i_ < n_ && s_[i_] != '"') {
      char c = s_[i_++];
      if (c != '\\') {
        out.push_back(c);
        continue;
      }
      if (i_ >= n_) return Fail("unterminated escape");
      char e = s_[i_++];
      switch (e) {
        case 'n': out.push_back('\n'); break;
        case 't': out.push_back('\t'); break;
        case 'r': out.push_back('\r'); break;
        case 'b': out.push_back('\b'); break;
        case 'f': out.push_back('\f'); break;
        case 'u': {
          if (i_ + 4 > n_) return Fail("bad \\u escape");
          unsigned cp = (unsigned)strtoul(std::string(s_ + i_, 4).c_str(), nullptr, 16);
          i_ += 4;
          if (cp < 0x80) {
            out.push_back((char)cp);
          } else if (cp < 0x800) {
            out.push_back((char)(0xC0 | (cp >> 6)));
            out.push_back((char)(0x80 | (cp & 0x3F)));
          } else {
            out.push_back((char)(0xE0 | (cp >> 12)));
            out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
            out.push_back((char)(0x80 | (cp & 0x3F)));
          }
          break;
        }
        default: out.push_back(e);
      }
    }
    if (i_ >= n_) return Fail("unterminated string");
    i_++;
    return true;
  }
  bool Value(Json& out, int depth) {
    if (depth > 512) return Fail("nesting too deep");
    SkipWs();
    if (i_ >= n_) return Fail("unexpected end of input");
    char c = s_[i_];
    if (c == '{') {
      i_++;
      out = Json::object();
      SkipWs();
      if (i_ < n_ && s_[i_] == '}') {
        i_++;
        return true;
      }
      while (true) {
        SkipWs();
        std::string key;
        if (!String(key)) return false;
        SkipWs();
        if (i_ >= n_ || s_[i_] != ':') return Fail("expected ':'");
        i_++;
        Json v;
        if (!Value(v, depth + 1)) return false;
        out.obj_.emplace_back(std::move(key), std::move(v));
        SkipWs();
        if (i_ < n_ && s_[i_] == ',') {
          i_++;
          continue;
        }
        if (i_ < n_ && s_[i_] == '}') {
          i_++;
          return true;
        }
        return Fail("expected ',' or '}'");
      }
    }
    if (c == '[') {
      i_++;
      out = Json::array();
      SkipWs();
      if (i_ < n_ && s_[i_] == ']') {
        i_++;
        return true;
      }
      while (true) {
        Json v;
        if (!Value(v, depth + 1)) return false;
        out.arr_.push_back(std::move(v));
        SkipWs();
        if (i_ < n_ && s_[i_] == ',') {
          i_++;
          continue;
        }
        if (i_ < n_ && s_[i_] == ']') {
          i_++;
          return true;
        }
        return Fail("expected ',' or ']'");
      }
    }
    if (c == '"') {
      out = Json::string("");
      return String(out.str_);
    }
    if (Lit("true")) {
      out = Json::boolean(true);
      return true;
    }
    if (Lit("false")) {
      out = Json::boolean(false);
      return true;
    }
    if (Lit("null")) {
      out = Json();
      return true;
    }
    size_t st = i_;
    if (i_ < n_ && (s_[i_] == '-' || s_[i_] == '+')) i_++;
    bool integral = true;
    while (i_ < n_ && (isdigit((unsigned char)s_[i_]) || s_[i_] == '.' || s_[i_] == 'e' || s_[i_] == 'E' ||
                       s_[i_] == '-' || s_[i_] == '+')) {
      if (s_[i_] == '.' || s_[i_] == 'e' || s_[i_] == 'E') integral = false;
      i_++;
    }
    if (i_ == st) return Fail("invalid value");
    std::string tok(s_ + st, i_ - st);
    char* end = nullptr;
    double v = strtod(tok.c_str(), &end);
    if (end == tok.c_str() || *end != 0) {
      i_ = st;
      return Fail("invalid number");
    }
    out = Json::number(v);
    out.integral_ = integral;
    return true;
  }
};

bool Json::Parse(const std::string& text, Json& out, std::string& err) {
  JsonParser p(text);
  return p.Run(out, err);
}

bool Json::ParseFile(const std::string& path, Json& out, std::string& err) {
  std::ifstream f(path, std::ios::binary);
  if (!f.is_open()) {
    err = "Failed to open json file: " + path;
    return false;
  }
  std::stringstream ss;
  ss << f.rdbuf();
  if (!Parse(ss.str(), out, err)) {
    err = path + ": " + err;
    return false;
  }
  return true;
}

const Json* Json::find(const std::string& key) const {
  if (type_ != Type::kObject) return nullptr;
  for (const auto& kv : obj_)
    if (kv.first == key) return &kv.second;
  return nullptr;
}

void Json::set(const std::string& key, Json v) {
  type_ = Type::kObject;
  for (auto& kv : obj_)
    if (kv.first == key) {
      kv.second = std::move(v);
      return;
    }
  obj_.emplace_back(key, std::move(v));
}

// Shortest round-trip decimal of v, laid out like nlohmann::json (grisu2 digits + format_buffer:
// fixed notation for decimal exponents in (-4, 15], "x.0" for integral values, else d.ddde+XX).
static std::string ShortestDouble(double v) {
  if (std::isnan(v) || std::isinf(v)) return "null";  // nlohmann writes null for non-finite
  if (v == 0.0) return std::signbit(v) ? "-0.0" : "0.0";
  char buf[64];
  int prec = 1;
  for (; prec <= 17; prec++) {
    snprintf(buf, sizeof(buf), "%.*e", prec - 1, v);
    if (strtod(buf, nullptr) == v) break;
  }
  std::string e(buf);
  bool neg = e[0] == '-';
  if (neg) e.erase(0, 1);
  size_t epos = e.find('e');
  int exp10 = atoi(e.c_str() + epos + 1);
  std::string digits;
  for (size_t k = 0; k < epos; k++)
    if (e[k] != '.') digits.push_back(e[k]);
  while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
  int len = (int)digits.size();
  int n = exp10 + 1;  // position of the decimal point relative to the digits
  std::string out;
  if (len <= n && n <= 15) {
    out = digits + std::string((size_t)(n - len), '0') + ".0";
  } else if (0 < n && n <= 15) {
    out = digits.substr(0, (size_t)n) + "." + digits.substr((size_t)n);
  } else if (-4 < n && n <= 0) {
    out = "0." + std::string((size_t)(-n), '0') + digits;
  } else {
    out = digits.substr(0, 1);
    if (len > 1) out += "." + digits.substr(1);
    char eb[16];
    snprintf(eb, sizeof(eb), "e%c%02d", n - 1 < 0 ? '-' : '+', std::abs(n - 1));
    out += eb;
  }
  return neg ? "-" + out : out;
}

void Json::DumpTo(std::string& out, int indent, int level) const {
  auto nl = [&](int lv) {
    out.push_back('\n');
    out.append((size_t)(indent * lv), ' ');
  };
  switch (type_) {
    case Type::kNull: out += "null"; break;
    case Type::kBool: out += bool_ ? "true" : "false"; break;
    case Type::kNumber:
      if (integral_) {
        out += std::to_string((long long)num_);
      } else {
        out += ShortestDouble(num_);
      }
      break;
    case Type::kString:
      out.push_back('"');
      for (char c : str_) {
        if (c == '"' || c == '\\') out.push_back('\\');
        out.push_back(c);
      }
      out.push_back('"');
      break;
    case Type::kArray:
      if (arr_.empty()) {
        out += "[]";
        break;
      }
      out.push_back('[');
      for (size_t k = 0; k < arr_.size(); k++) {
        nl(level + 1);
        arr_[k].DumpTo(out, indent, level + 1);
        if (k + 1 < arr_.size()) out.push_back(',');
      }
      nl(level);
      out.push_back(']');
      break;
    case Type::kObject: {
      if (obj_.empty()) {
        out += "{}";
        break;
      }
      std::vector<const std::pair<std::string, Json>*> sorted;
      for (const auto& kv : obj_) sorted.push_back(&kv);
      std::sort(sorted.begin(), sorted.end(), [](auto* a, auto* b) { return a->first < b->first; });
      out.push_back('{');
      for (size_t k = 0; k < sorted.size(); k++) {
        nl(level + 1);
        out += "\"" + sorted[k]->first + "\": ";
        sorted[k]->second.DumpTo(out, indent, level + 1);
        if (k + 1 < sorted.size()) out.push_back(',');
      }
      nl(level);
      out.push_back('}');
      break;
    }
  }
}

std::string Json::Dump(int indent) const {
  std::string out;
  DumpTo(out, indent, 0);
  return out;
}

}  // namespace rt2
