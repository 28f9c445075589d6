// value.cpp — JSON / YAML-subset parsing, serialisation, RFC 7386 / RFC 6902
// patching and Kubernetes quantities for the host side of ccka.
//
// The YAML subset covers what the reference's manifests use
// (demo_30_burst_configure.sh:78-141, demo_10_setup_configure.sh and the
// RBAC heredocs): block mappings and sequences (including the "indentless"
// sequences kubectl manifests use under a key), "- key: v" sequence items,
// plain / single / double quoted scalars, flow [..] / {..} collections,
// comments, and multi-document streams separated by ---.
#include "value.h"

#include <cctype>
#include <cmath>
#include <cstdlib>
#include <cstring>

namespace ccka::host {

// ------------------------------------------------------------------ Value
const Value* Value::get(const std::string& k) const {
  if (kind != Map) return nullptr;
  for (auto& kv : map)
    if (kv.first == k) return &kv.second;
  return nullptr;
}
Value* Value::get(const std::string& k) {
  if (kind != Map) return nullptr;
  for (auto& kv : map)
    if (kv.first == k) return &kv.second;
  return nullptr;
}
Value& Value::set(const std::string& k, Value v) {
  if (kind != Map) { *this = object(); }
  for (auto& kv : map)
    if (kv.first == k) { kv.second = std::move(v); return kv.second; }
  map.emplace_back(k, std::move(v));
  return map.back().second;
}
bool Value::erase(const std::string& k) {
  if (kind != Map) return false;
  for (size_t i = 0; i < map.size(); ++i)
    if (map[i].first == k) { map.erase(map.begin() + (long)i); return true; }
  return false;
}
const Value* Value::at(const std::vector<std::string>& path) const {
  const Value* v = this;
  for (auto& p : path) {
    if (!v) return nullptr;
    if (v->kind == Seq) {
      char* end = nullptr;
      long idx = std::strtol(p.c_str(), &end, 10);
      if (*end || idx < 0 || (size_t)idx >= v->seq.size()) return nullptr;
      v = &v->seq[(size_t)idx];
    } else {
      v = v->get(p);
    }
  }
  return v;
}
std::string Value::as_string(const std::string& dflt) const {
  if (kind == Null || kind == Seq || kind == Map) return dflt;
  return text;
}
int64_t Value::as_int(int64_t dflt) const {
  if (!is_scalar()) return dflt;
  char* end = nullptr;
  long long x = std::strtoll(text.c_str(), &end, 10);
  if (end == text.c_str()) return dflt;
  return x;
}

// ------------------------------------------------------------------ scalars
static bool looks_number(const std::string& s) {
  if (s.empty()) return false;
  size_t i = 0;
  if (s[i] == '-' || s[i] == '+') ++i;
  bool digit = false, dot = false, exp = false;
  for (; i < s.size(); ++i) {
    const char c = s[i];
    if (std::isdigit((unsigned char)c)) digit = true;
    else if (c == '.' && !dot && !exp) dot = true;
    else if ((c == 'e' || c == 'E') && digit && !exp) {
      exp = true;
      if (i + 1 < s.size() && (s[i + 1] == '-' || s[i + 1] == '+')) ++i;
      if (i + 1 >= s.size()) return false;  // "1e", "1e+": no exponent digits
    } else return false;
  }
  return digit;
}

static Value plain_scalar(const std::string& s) {
  if (s.empty() || s == "~" || s == "null" || s == "Null" || s == "NULL") return Value();
  if (s == "true" || s == "True" || s == "TRUE" || s == "false" || s == "False" || s == "FALSE") {
    Value v;
    v.kind = Value::Bool;
    v.text = (s[0] == 't' || s[0] == 'T') ? "true" : "false";
    return v;
  }
  if (looks_number(s)) return Value::num(s);
  return Value::str(s, false);
}

static std::string trim(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && std::isspace((unsigned char)s[a])) ++a;
  while (b > a && std::isspace((unsigned char)s[b - 1])) --b;
  return s.substr(a, b - a);
}

// ------------------------------------------------------------------ JSON
namespace {
struct JsonParser {
  const std::string& s;
  size_t i = 0;
  explicit JsonParser(const std::string& x) : s(x) {}
  [[noreturn]] void err(const char* what) {
    throw ParseError(std::string("json: ") + what + " at offset " + std::to_string(i));
  }
  void ws() {
    while (i < s.size() && std::isspace((unsigned char)s[i])) ++i;
  }
  static void utf8(std::string& out, unsigned cp) {
    if (cp < 0x80) out += (char)cp;
    else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 63)); }
    else if (cp < 0x10000) {
      out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 63)); out += (char)(0x80 | (cp & 63));
    } else {
      out += (char)(0xF0 | (cp >> 18)); out += (char)(0x80 | ((cp >> 12) & 63));
      out += (char)(0x80 | ((cp >> 6) & 63)); out += (char)(0x80 | (cp & 63));
    }
  }
  unsigned hex(int n) {
    if (i + (size_t)n > s.size()) err("bad hex escape");
    unsigned v = 0;
    for (int d = 0; d < n; ++d) {
      const char h = s[i++];
      v <<= 4;
      if (h >= '0' && h <= '9') v |= (unsigned)(h - '0');
      else if (h >= 'a' && h <= 'f') v |= (unsigned)(h - 'a' + 10);
      else if (h >= 'A' && h <= 'F') v |= (unsigned)(h - 'A' + 10);
      else err("bad hex escape");
    }
    return v;
  }
  // a double-quoted string; `yaml` adds YAML 1.1's extra escapes (\0 \a \v \e
  // \xHH \UHHHHHHHH \N \_ \L \P, escaped space) to JSON's
  std::string str(bool yaml = false) {
    if (s[i] != '"') err("expected string");
    ++i;
    std::string out;
    while (i < s.size() && s[i] != '"') {
      char c = s[i++];
      if (c == '\\') {
        if (i >= s.size()) err("bad escape");
        char e = s[i++];
        switch (e) {
          case 'n': out += '\n'; break;
          case 't': out += '\t'; break;
          case 'r': out += '\r'; break;
          case 'b': out += '\b'; break;
          case 'f': out += '\f'; break;
          case '"': case '\\': case '/': out += e; break;
          case 'u': {
            unsigned cp = hex(4);
            if (cp >= 0xD800 && cp < 0xDC00 && i + 6 <= s.size() && s[i] == '\\' && s[i + 1] == 'u') {
              const size_t save = i;
              i += 2;
              const unsigned lo = hex(4);
              if (lo >= 0xDC00 && lo < 0xE000) cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
              else i = save;
            }
            utf8(out, cp);
            break;
          }
          default:
            if (!yaml) err("bad escape");
            switch (e) {
              case '0': out += '\0'; break;
              case 'a': out += '\a'; break;
              case 'v': out += '\v'; break;
              case 'e': out += '\x1b'; break;
              case ' ': case '\t': out += e; break;
              case 'x': utf8(out, hex(2)); break;
              case 'U': utf8(out, hex(8)); break;
              case 'N': utf8(out, 0x85); break;
              case '_': utf8(out, 0xA0); break;
              case 'L': utf8(out, 0x2028); break;
              case 'P': utf8(out, 0x2029); break;
              default: err("bad escape");
            }
        }
      } else {
        out += c;
      }
    }
    if (i >= s.size()) err("unterminated string");
    ++i;
    return out;
  }
  Value val() {
    ws();
    if (i >= s.size()) err("unexpected end");
    const char c = s[i];
    if (c == '{') {
      ++i;
      Value m = Value::object();
      ws();
      if (s[i] == '}') { ++i; return m; }
      for (;;) {
        ws();
        std::string k = str();
        ws();
        if (s[i] != ':') err("expected ':'");
        ++i;
        m.map.emplace_back(k, val());
        ws();
        if (s[i] == ',') { ++i; continue; }
        if (s[i] == '}') { ++i; return m; }
        err("expected ',' or '}'");
      }
    }
    if (c == '[') {
      ++i;
      Value a = Value::array();
      ws();
      if (s[i] == ']') { ++i; return a; }
      for (;;) {
        a.seq.push_back(val());
        ws();
        if (s[i] == ',') { ++i; continue; }
        if (s[i] == ']') { ++i; return a; }
        err("expected ',' or ']'");
      }
    }
    if (c == '"') return Value::str(str());
    size_t j = i;
    while (j < s.size() && !std::strchr(",]} \t\r\n", s[j])) ++j;
    std::string tok = s.substr(i, j - i);
    i = j;
    if (tok == "null") return Value();
    if (tok == "true" || tok == "false") {
      Value v;
      v.kind = Value::Bool;
      v.text = tok;
      return v;
    }
    if (looks_number(tok)) return Value::num(tok);
    err("bad token");
  }
};
}  // namespace

Value parse_json(const std::string& text) {
  JsonParser p(text);
  Value v = p.val();
  p.ws();
  if (p.i != text.size()) p.err("trailing characters");
  return v;
}

static void json_escape(std::string& o, const std::string& s) {
  o += '"';
  for (char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\t': o += "\\t"; break;
      case '\r': o += "\\r"; break;
      default:
        if ((unsigned char)c < 0x20) {
          char b[8];
          std::snprintf(b, sizeof b, "\\u%04x", c);
          o += b;
        } else {
          o += c;
        }
    }
  }
  o += '"';
}

static void to_json_rec(std::string& o, const Value& v) {
  switch (v.kind) {
    case Value::Null: o += "null"; break;
    case Value::Bool:
    case Value::Number: o += v.text; break;
    case Value::String: json_escape(o, v.text); break;
    case Value::Seq:
      o += '[';
      for (size_t k = 0; k < v.seq.size(); ++k) {
        if (k) o += ',';
        to_json_rec(o, v.seq[k]);
      }
      o += ']';
      break;
    case Value::Map:
      o += '{';
      for (size_t k = 0; k < v.map.size(); ++k) {
        if (k) o += ',';
        json_escape(o, v.map[k].first);
        o += ':';
        to_json_rec(o, v.map[k].second);
      }
      o += '}';
      break;
  }
}

std::string to_json(const Value& v) {
  std::string o;
  to_json_rec(o, v);
  return o;
}

// ------------------------------------------------------------------ YAML
namespace {
struct Line {
  int indent;
  std::string text;
  int no;
};

// YAML quotes and flow brackets only open at the start of a scalar: after
// nothing, an open bracket or comma of an enclosing flow collection, or a
// ': ' / '- ' / '? ' indicator. Anywhere else ("0\"", "a[0]", "it's") they
// are plain characters. Calls f(k, depth) for every character outside quotes
// (depth = open flow brackets); f returns true to stop the scan. Returns the
// quote character when the text ends inside a quoted scalar (it continues on
// the next line), else 0.
template <class F>
static char yaml_scan(const std::string& s, F&& f) {
  int depth = 0;
  auto token_start = [&](size_t k, auto&& self) -> bool {
    size_t p = k;
    while (p > 0 && (s[p - 1] == ' ' || s[p - 1] == '\t')) --p;
    if (p == 0) return true;
    const char c = s[p - 1];
    if (c == '[' || c == '{') return depth > 0;
    if (c == ',') return depth > 0;
    if ((c == ':' || c == '-' || c == '?') && p < k) return c == ':' || self(p - 1, self);
    return false;
  };
  for (size_t k = 0; k < s.size(); ++k) {
    const char c = s[k];
    if ((c == '\'' || c == '"') && token_start(k, token_start)) {
      size_t j = k + 1;
      for (; j < s.size(); ++j) {
        if (c == '"' && s[j] == '\\') { ++j; continue; }
        if (s[j] == c) {
          if (c == '\'' && j + 1 < s.size() && s[j + 1] == '\'') { ++j; continue; }
          break;
        }
      }
      if (j >= s.size()) return c;  // unterminated: continues on the next line
      k = j;  // the closing quote
      continue;
    }
    if (c == '[' || c == '{') {
      if (depth > 0 || token_start(k, token_start)) ++depth;
    } else if ((c == ']' || c == '}') && depth > 0) {
      --depth;
    }
    if (f(k, depth)) return 0;
  }
  return 0;
}

static char open_quote(const std::string& s) {
  return yaml_scan(s, [](size_t, int) { return false; });
}

std::string strip_comment(const std::string& s) {
  size_t cut = std::string::npos;
  yaml_scan(s, [&](size_t k, int) {
    if (s[k] == '#' && (k == 0 || std::isspace((unsigned char)s[k - 1]))) { cut = k; return true; }
    return false;
  });
  return cut == std::string::npos ? s : s.substr(0, cut);
}

// position of the ':' that ends a mapping key, or npos
size_t key_colon(const std::string& s) {
  if (!s.empty() && (s[0] == '[' || s[0] == '{')) return std::string::npos;  // flow collection scalar
  size_t at = std::string::npos;
  yaml_scan(s, [&](size_t k, int depth) {
    if (s[k] == ':' && depth == 0 && (k + 1 == s.size() || s[k + 1] == ' ' || s[k + 1] == '\t')) { at = k; return true; }
    return false;
  });
  return at;
}

bool is_dash(const std::string& s) { return s == "-" || (s.size() >= 2 && s[0] == '-' && s[1] == ' '); }

struct FlowParser {
  const std::string& s;
  size_t i = 0;
  int no;
  FlowParser(const std::string& x, int line) : s(x), no(line) {}
  [[noreturn]] void err(const char* w) {
    throw ParseError("yaml line " + std::to_string(no) + ": " + w);
  }
  void ws() {
    while (i < s.size() && std::isspace((unsigned char)s[i])) ++i;
  }
  Value scalar() {
    ws();
    if (i < s.size() && s[i] == '"') {
      JsonParser jp(s);
      jp.i = i;
      std::string t = jp.str(true);
      i = jp.i;
      return Value::str(t);
    }
    if (i < s.size() && s[i] == '\'') {
      ++i;
      std::string t;
      while (i < s.size()) {
        if (s[i] == '\'') {
          if (i + 1 < s.size() && s[i + 1] == '\'') { t += '\''; i += 2; continue; }
          break;
        }
        t += s[i++];
      }
      if (i >= s.size()) err("unterminated quote");
      ++i;
      return Value::str(t);
    }
    size_t j = i;
    while (j < s.size() && !std::strchr(",]}", s[j]) && !(s[j] == ':' && (j + 1 == s.size() || s[j + 1] == ' ')))
      ++j;
    std::string tok = trim(s.substr(i, j - i));
    i = j;
    return plain_scalar(tok);
  }
  Value val() {
    ws();
    if (i < s.size() && s[i] == '[') {
      ++i;
      Value a = Value::array();
      ws();
      if (i < s.size() && s[i] == ']') { ++i; return a; }
      for (;;) {
        a.seq.push_back(val());
        ws();
        if (i < s.size() && s[i] == ',') { ++i; ws(); if (i < s.size() && s[i] == ']') { ++i; return a; } continue; }
        if (i < s.size() && s[i] == ']') { ++i; return a; }
        err("bad flow sequence");
      }
    }
    if (i < s.size() && s[i] == '{') {
      ++i;
      Value m = Value::object();
      ws();
      if (i < s.size() && s[i] == '}') { ++i; return m; }
      for (;;) {
        Value k = scalar();
        ws();
        if (i >= s.size() || s[i] != ':') err("expected ':' in flow mapping");
        ++i;
        m.map.emplace_back(k.text, val());
        ws();
        if (i < s.size() && s[i] == ',') { ++i; continue; }
        if (i < s.size() && s[i] == '}') { ++i; return m; }
        err("bad flow mapping");
      }
    }
    return scalar();
  }
};

Value inline_value(const std::string& raw, int no) {
  const std::string s = trim(raw);
  FlowParser fp(s, no);
  Value v = fp.val();
  fp.ws();
  if (fp.i != s.size()) {
    // a plain scalar containing flow characters: keep the text
    return plain_scalar(s);
  }
  return v;
}

struct YamlParser {
  std::vector<Line>& L;
  size_t pos = 0;
  explicit YamlParser(std::vector<Line>& l) : L(l) {}

  Value block(int indent) {
    if (pos >= L.size() || L[pos].indent < indent) return Value();
    const Line& ln = L[pos];
    if (is_dash(ln.text)) return seq(ln.indent);
    if (key_colon(ln.text) != std::string::npos) return mapping(ln.indent);
    ++pos;
    return inline_value(ln.text, ln.no);
  }

  Value block_scalar(int parent_indent, bool literal) {
    std::string out;
    int ind = -1;
    while (pos < L.size() && L[pos].indent > parent_indent) {
      if (ind < 0) ind = L[pos].indent;
      out += std::string((size_t)(L[pos].indent - ind), ' ') + L[pos].text + (literal ? "\n" : " ");
      ++pos;
    }
    return Value::str(out);
  }

  Value mapping(int indent) {
    Value m = Value::object();
    while (pos < L.size() && L[pos].indent == indent && !is_dash(L[pos].text)) {
      const Line ln = L[pos];
      const size_t c = key_colon(ln.text);
      if (c == std::string::npos) throw ParseError("yaml line " + std::to_string(ln.no) + ": expected 'key:'");
      std::string key = trim(ln.text.substr(0, c));
      if (key.size() >= 2 && (key[0] == '"' || key[0] == '\'')) key = inline_value(key, ln.no).text;
      const std::string rest = trim(ln.text.substr(c + 1));
      ++pos;
      Value v;
      if (rest.empty()) {
        if (pos < L.size() && (L[pos].indent > indent || (L[pos].indent == indent && is_dash(L[pos].text))))
          v = block(L[pos].indent);
      } else if (rest[0] == '|' || rest[0] == '>') {
        v = block_scalar(indent, rest[0] == '|');
      } else {
        v = inline_value(rest, ln.no);
      }
      m.map.emplace_back(key, std::move(v));
    }
    return m;
  }

  Value seq(int indent) {
    Value a = Value::array();
    while (pos < L.size() && L[pos].indent == indent && is_dash(L[pos].text)) {
      Line& ln = L[pos];
      std::string rest = ln.text.size() > 1 ? ln.text.substr(1) : "";
      size_t sp = 0;
      while (sp < rest.size() && rest[sp] == ' ') ++sp;
      rest = rest.substr(sp);
      if (rest.empty()) {
        ++pos;
        a.seq.push_back(pos < L.size() && L[pos].indent > indent ? block(L[pos].indent) : Value());
      } else if (is_dash(rest) || key_colon(rest) != std::string::npos) {
        // the item starts on the dash line: re-read that line as a nested block
        ln.indent = indent + 1 + (int)sp;
        ln.text = rest;
        a.seq.push_back(block(ln.indent));
      } else {
        ++pos;
        a.seq.push_back(inline_value(rest, ln.no));
      }
    }
    return a;
  }
};
}  // namespace

// bracket depth of a flow collection's text (quotes skipped): > 0 while it
// continues on the next line (emitters wrap long flow collections)
static int flow_depth(const std::string& s) {
  int depth = 0;
  yaml_scan(s, [&](size_t, int d) { depth = d; return false; });
  return depth;
}

// the value part of a block line that starts a flow collection, else ""
static std::string flow_start(const std::string& t) {
  std::string v;
  if (!t.empty() && (t[0] == '[' || t[0] == '{')) v = t;
  else if (is_dash(t)) v = trim(t.substr(1));
  else {
    const size_t c = key_colon(t);
    if (c != std::string::npos) v = trim(t.substr(c + 1));
  }
  if (!v.empty() && (v[0] == '[' || v[0] == '{')) return v;
  if (is_dash(t) && !v.empty() && v != t) return flow_start(v);  // "- key: [..." or "- - [..."
  return std::string();
}

std::vector<Value> parse_yaml_documents(const std::string& text) {
  std::vector<std::vector<Line>> docs(1);
  size_t start = 0;
  int no = 0;
  int pend_depth = 0;  // open brackets of a flow collection continued on the next line
  char pend_quote = 0;  // quote of a quoted scalar continued on the next line
  int pend_blank = 0;   // empty lines inside that scalar so far
  while (start <= text.size()) {
    size_t end = text.find('\n', start);
    if (end == std::string::npos) end = text.size();
    std::string raw = text.substr(start, end - start);
    start = end + 1;
    ++no;
    if (!raw.empty() && raw.back() == '\r') raw.pop_back();
    if (raw.find('\t') != std::string::npos && raw.find_first_not_of(" \t") != std::string::npos &&
        raw[raw.find_first_not_of(' ')] == '\t')
      throw ParseError("yaml line " + std::to_string(no) + ": tab indentation");
    if (pend_quote) {  // line folding inside a multi-line quoted scalar (YAML 1.1 7.3)
      const std::string t = trim(raw);
      if (t.empty()) {
        ++pend_blank;
        if (end == text.size()) break;
        continue;
      }
      std::string& acc = docs.back().back().text;
      size_t bs = 0;
      while (bs < acc.size() && acc[acc.size() - 1 - bs] == '\\') ++bs;
      if (pend_quote == '"' && (bs & 1)) {  // escaped line break: joined without a space
        acc.pop_back();
        acc += std::string((size_t)pend_blank, '\n');
      } else {
        while (!acc.empty() && (acc.back() == ' ' || acc.back() == '\t')) acc.pop_back();
        acc += pend_blank ? std::string((size_t)pend_blank, '\n') : std::string(" ");
      }
      pend_blank = 0;
      acc += t;
      pend_quote = open_quote(acc);
      if (!pend_quote) {
        acc = trim(strip_comment(acc));
        const std::string fv = flow_start(acc);
        pend_depth = fv.empty() ? 0 : std::max(0, flow_depth(fv));
      }
      if (end == text.size()) break;
      continue;
    }
    const std::string body = strip_comment(raw);
    const std::string t = trim(body);
    if (pend_depth > 0 && !t.empty()) {  // continuation of a wrapped flow collection
      docs.back().back().text += " " + t;
      pend_depth = std::max(0, flow_depth(flow_start(docs.back().back().text)));
      pend_quote = open_quote(docs.back().back().text);
      if (end == text.size()) break;
      continue;
    }
    if (t.empty()) { if (end == text.size()) break; continue; }
    if (t == "---" || t.rfind("--- ", 0) == 0) { docs.emplace_back(); continue; }
    if (t == "...") continue;
    int ind = 0;
    while (ind < (int)body.size() && body[(size_t)ind] == ' ') ++ind;
    docs.back().push_back({ind, trim(body), no});
    const std::string fv = flow_start(docs.back().back().text);
    if (!fv.empty()) pend_depth = std::max(0, flow_depth(fv));
    pend_quote = open_quote(docs.back().back().text);
    if (end == text.size()) break;
  }
  std::vector<Value> out;
  for (auto& d : docs) {
    if (d.empty()) continue;
    YamlParser p(d);
    Value v = p.block(d[0].indent);
    if (p.pos != d.size())
      throw ParseError("yaml line " + std::to_string(d[p.pos].no) + ": unexpected indentation");
    out.push_back(std::move(v));
  }
  return out;
}

// ------------------------------------------------------------------ patches
void apply_merge_patch(Value& target, const Value& patch) {
  if (!patch.is_map()) { target = patch; return; }
  if (!target.is_map()) target = Value::object();
  for (auto& kv : patch.map) {
    if (kv.second.kind == Value::Null) {
      target.erase(kv.first);
    } else {
      Value* cur = target.get(kv.first);
      if (!cur) cur = &target.set(kv.first, Value());
      apply_merge_patch(*cur, kv.second);
    }
  }
}

static std::vector<std::string> split_pointer(const std::string& ptr) {
  std::vector<std::string> out;
  if (ptr.empty()) return out;
  if (ptr[0] != '/') throw ParseError("json patch: bad pointer " + ptr);
  size_t k = 1;
  for (;;) {
    size_t e = ptr.find('/', k);
    std::string tok = ptr.substr(k, e == std::string::npos ? std::string::npos : e - k);
    std::string dec;
    for (size_t j = 0; j < tok.size(); ++j) {
      if (tok[j] == '~' && j + 1 < tok.size()) { dec += tok[j + 1] == '1' ? '/' : '~'; ++j; }
      else dec += tok[j];
    }
    out.push_back(dec);
    if (e == std::string::npos) break;
    k = e + 1;
  }
  return out;
}

void apply_json_patch(Value& target, const Value& patch) {
  if (!patch.is_seq()) throw ParseError("json patch: document is not an array");
  for (auto& op : patch.seq) {
    const Value* o = op.get("op");
    const Value* path = op.get("path");
    if (!o || !path) throw ParseError("json patch: operation needs op and path");
    const std::string name = o->as_string();
    auto toks = split_pointer(path->as_string());
    if (toks.empty()) throw ParseError("json patch: root replacement not supported");
    Value* parent = &target;
    for (size_t k = 0; k + 1 < toks.size(); ++k) {
      Value* nx = nullptr;
      if (parent->is_map()) nx = parent->get(toks[k]);
      else if (parent->is_seq()) {
        char* end = nullptr;
        long idx = std::strtol(toks[k].c_str(), &end, 10);
        if (!*end && idx >= 0 && (size_t)idx < parent->seq.size()) nx = &parent->seq[(size_t)idx];
      }
      if (!nx)
        throw ParseError("jsonpatch " + name + " operation does not apply: doc is missing path: " + path->as_string());
      parent = nx;
    }
    const std::string& last = toks.back();
    const Value* val = op.get("value");
    if (name == "add" || name == "replace") {
      if (!val) throw ParseError("json patch: " + name + " needs a value");
      if (parent->is_map()) {
        if (name == "replace" && !parent->get(last))
          throw ParseError("jsonpatch replace operation does not apply: doc is missing key: " + path->as_string());
        parent->set(last, *val);
      } else if (parent->is_seq()) {
        if (last == "-" && name == "add") { parent->seq.push_back(*val); continue; }
        char* end = nullptr;
        long idx = std::strtol(last.c_str(), &end, 10);
        if (*end || idx < 0 || (size_t)idx > parent->seq.size() || (name == "replace" && (size_t)idx == parent->seq.size()))
          throw ParseError("json patch: index out of range: " + path->as_string());
        if (name == "add") parent->seq.insert(parent->seq.begin() + idx, *val);
        else parent->seq[(size_t)idx] = *val;
      } else {
        throw ParseError("jsonpatch " + name + " operation does not apply: doc is missing path: " + path->as_string());
      }
    } else if (name == "remove") {
      if (parent->is_map()) {
        if (!parent->erase(last)) throw ParseError("jsonpatch remove operation does not apply: doc is missing key: " + path->as_string());
      } else if (parent->is_seq()) {
        long idx = std::strtol(last.c_str(), nullptr, 10);
        if (idx < 0 || (size_t)idx >= parent->seq.size()) throw ParseError("json patch: index out of range");
        parent->seq.erase(parent->seq.begin() + idx);
      }
    } else if (name == "test") {
      const Value* cur = parent->is_map() ? parent->get(last) : nullptr;
      if (!cur || !val || to_json(*cur) != to_json(*val)) throw ParseError("json patch: test failed at " + path->as_string());
    } else {
      throw ParseError("json patch: unsupported op " + name);
    }
  }
}

// ------------------------------------------------------------------ quantities
static double parse_decimal(const std::string& s, size_t* used) {
  char* end = nullptr;
  const double v = std::strtod(s.c_str(), &end);
  *used = (size_t)(end - s.c_str());
  return v;
}

int64_t cpu_millis(const std::string& q0) {
  const std::string q = trim(q0);
  size_t u = 0;
  const double v = parse_decimal(q, &u);
  const std::string suf = q.substr(u);
  if (u == 0) throw ParseError("bad cpu quantity: " + q0);
  if (suf == "m") return (int64_t)std::ceil(v);
  if (suf.empty()) return (int64_t)std::ceil(v * 1000.0 - 1e-9);
  throw ParseError("bad cpu quantity: " + q0);
}

int64_t mem_mib(const std::string& q0) {
  const std::string q = trim(q0);
  size_t u = 0;
  const double v = parse_decimal(q, &u);
  const std::string suf = q.substr(u);
  if (u == 0) throw ParseError("bad memory quantity: " + q0);
  double bytes;
  if (suf.empty()) bytes = v;
  else if (suf == "Ki") bytes = v * 1024.0;
  else if (suf == "Mi") bytes = v * 1048576.0;
  else if (suf == "Gi") bytes = v * 1073741824.0;
  else if (suf == "Ti") bytes = v * 1099511627776.0;
  else if (suf == "k") bytes = v * 1e3;
  else if (suf == "M") bytes = v * 1e6;
  else if (suf == "G") bytes = v * 1e9;
  else if (suf == "T") bytes = v * 1e12;
  else throw ParseError("bad memory quantity: " + q0);
  return (int64_t)std::ceil(bytes / 1048576.0 - 1e-9);
}

int64_t duration_s(const std::string& q0) {
  const std::string q = trim(q0);
  if (q == "Never") return (int64_t)1 << 30;
  int64_t total = 0;
  size_t k = 0;
  bool any = false;
  while (k < q.size()) {
    size_t u = 0;
    const double v = parse_decimal(q.substr(k), &u);
    if (u == 0) throw ParseError("bad duration: " + q0);
    k += u;
    std::string unit;
    while (k < q.size() && std::isalpha((unsigned char)q[k])) unit += q[k++];
    double mul;
    if (unit == "s") mul = 1;
    else if (unit == "m") mul = 60;
    else if (unit == "h") mul = 3600;
    else if (unit == "ms") mul = 1e-3;
    else throw ParseError("bad duration: " + q0);
    total += (int64_t)std::llround(v * mul);
    any = true;
  }
  if (!any) throw ParseError("bad duration: " + q0);
  return total;
}

}  // namespace ccka::host
