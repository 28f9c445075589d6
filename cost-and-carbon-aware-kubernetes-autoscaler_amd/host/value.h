// value.h — a small JSON/YAML document tree for Kubernetes manifests.
//
// The reference hands kubectl YAML manifests (demo_30_burst_configure.sh:78-141,
// demo_10_setup_configure.sh:162-210 of the captured run) and JSON / merge
// patches (demo_20_offpeak_configure.sh:59-81). This is the minimal document
// model the host needs to ingest and patch them: ordered maps (key order is
// preserved so re-serialisation is stable), sequences and scalars that keep
// their source spelling (numbers stay text until a typed accessor reads them).
#pragma once

#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace ccka::host {

struct ParseError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

struct Value {
  enum Kind { Null, Bool, Number, String, Seq, Map };
  Kind kind = Null;
  std::string text;  // Bool/Number/String scalar text
  bool quoted = false;
  std::vector<Value> seq;
  std::vector<std::pair<std::string, Value>> map;

  static Value str(std::string s, bool q = true) {
    Value v;
    v.kind = String;
    v.text = std::move(s);
    v.quoted = q;
    return v;
  }
  static Value num(std::string s) {
    Value v;
    v.kind = Number;
    v.text = std::move(s);
    return v;
  }
  static Value object() {
    Value v;
    v.kind = Map;
    return v;
  }
  static Value array() {
    Value v;
    v.kind = Seq;
    return v;
  }
  bool is_map() const { return kind == Map; }
  bool is_seq() const { return kind == Seq; }
  bool is_scalar() const { return kind == Bool || kind == Number || kind == String; }

  const Value* get(const std::string& k) const;
  Value* get(const std::string& k);
  Value& set(const std::string& k, Value v);
  bool erase(const std::string& k);
  // dotted path lookup ("spec.template.spec.nodeSelector"); keys containing
  // dots are addressed with a path vector instead
  const Value* at(const std::vector<std::string>& path) const;
  std::string as_string(const std::string& dflt = "") const;
  int64_t as_int(int64_t dflt = 0) const;
};

Value parse_json(const std::string& text);
std::vector<Value> parse_yaml_documents(const std::string& text);
std::string to_json(const Value& v);

// RFC 7386 merge patch (kubectl patch --type=merge)
void apply_merge_patch(Value& target, const Value& patch);
// RFC 6902 JSON patch (kubectl patch --type=json); throws ParseError with a
// kubectl-like message when a path does not exist
void apply_json_patch(Value& target, const Value& patch);

// Kubernetes quantities
int64_t cpu_millis(const std::string& q);  // "200m" -> 200, "1" -> 1000, "0.5" -> 500
int64_t mem_mib(const std::string& q);     // "128Mi" -> 128, "1Gi" -> 1024, "512M" -> 489 (ceil)
int64_t duration_s(const std::string& q);  // "30s" -> 30, "2m" -> 120, "1h" -> 3600

}  // namespace ccka::host
