// intern.cpp — the interning of SURVEY.md §8b(4) behind the C ABI (ca_intern_*, casim.h).
//
// A cgo shim turns API objects into the records' ids and bitsets: NoSchedule/NoExecute
// taints into taint classes and tolerations into masks over them
// (V/k8s.io/component-helpers/scheduling/corev1/helpers.go:63-101, V/k8s.io/api/core/v1/
// toleration.go:38-57), label pairs / keys / Gt-Lt keys referenced by selectors into
// bitsets and requirement rows (V/k8s.io/component-helpers/scheduling/corev1/nodeaffinity/
// nodeaffinity.go:223-293, V/k8s.io/apimachinery/pkg/labels/selector.go:223-267), host
// ports into triples with the 0.0.0.0 wildcard expanded (SF/types.go:887-931), scalar
// resources (V/k8s.io/kubernetes/pkg/scheduler/util/utils.go:158-161, SF/plugins/
// noderesources/fit.go:160-176) and node names into ids.  Host-only code; restates
// autoscaler_amd/intern.py, and both are pinned by tests/golden/intern_fixtures.json
// (tests/c_abi/intern_driver.c replays tests/golden/intern_calls.txt, derived from it).
#include <cstdint>
#include <cstring>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "casim.h"

namespace {

// a universe of values interned to bit positions, at most `cap` of them; a value past the
// width is remembered as overflow and has no id (intern.py:_Universe)
struct Universe {
    int32_t cap = 0;
    std::unordered_map<std::string, int32_t> ids;
    std::vector<std::string> keys;                 // by id
    std::unordered_set<std::string> overflow;
    explicit Universe(int32_t c) : cap(c) {}
    int32_t get(const std::string& k, bool create) {
        auto it = ids.find(k);
        if (it != ids.end()) return it->second;
        if (!create) return -1;
        if ((int32_t)ids.size() >= cap || overflow.count(k)) {
            overflow.insert(k);
            return -1;
        }
        const int32_t i = (int32_t)ids.size();
        ids.emplace(k, i);
        keys.push_back(k);
        return i;
    }
};

std::string s_or(const char* s) { return s ? std::string(s) : std::string(); }

// tuple keys: fields joined by a separator no API string contains
std::string key2(const std::string& a, const std::string& b) { return a + '\x1f' + b; }
std::string key3(const std::string& a, const std::string& b, const std::string& c) { return a + '\x1f' + b + '\x1f' + c; }

void split3(const std::string& k, std::string& a, std::string& b, std::string& c) {
    const size_t p = k.find('\x1f'), q = k.find('\x1f', p + 1);
    a = k.substr(0, p);
    b = k.substr(p + 1, q - p - 1);
    c = k.substr(q + 1);
}

bool alnum(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9'); }

// ^([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9]$ (validation.qualifiedNameFmt / label values)
bool name_fmt(const std::string& s) {
    if (s.empty() || !alnum(s.front()) || !alnum(s.back())) return false;
    for (char c : s)
        if (!alnum(c) && c != '-' && c != '_' && c != '.') return false;
    return true;
}

// DNS-1123 subdomain: dot-separated labels of [a-z0-9] with inner '-'
bool dns1123_subdomain(const std::string& s) {
    if (s.empty()) return false;
    size_t i = 0;
    while (true) {
        const size_t j = s.find('.', i);
        const std::string lab = s.substr(i, j == std::string::npos ? std::string::npos : j - i);
        if (lab.empty()) return false;
        auto lower_alnum = [](char c) { return (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'); };
        if (!lower_alnum(lab.front()) || !lower_alnum(lab.back())) return false;
        for (char c : lab)
            if (!lower_alnum(c) && c != '-') return false;
        if (j == std::string::npos) return true;
        i = j + 1;
    }
}

// validation.IsQualifiedName (apimachinery/pkg/util/validation)
bool qualified_name(const std::string& s) {
    std::string name;
    const size_t p = s.find('/');
    if (p == std::string::npos) {
        name = s;
    } else {
        if (s.find('/', p + 1) != std::string::npos) return false;
        const std::string prefix = s.substr(0, p);
        if (prefix.empty() || prefix.size() > 253 || !dns1123_subdomain(prefix)) return false;
        name = s.substr(p + 1);
    }
    return !name.empty() && name.size() <= 63 && name_fmt(name);
}

bool label_value(const std::string& v) { return v.empty() || (v.size() <= 63 && name_fmt(v)); }

// strconv.ParseInt(s, 10, 64): optional sign, decimal digits, in range
bool parse_int64(const std::string& s, int64_t* out) {
    size_t i = 0;
    bool neg = false;
    if (i < s.size() && (s[i] == '+' || s[i] == '-')) { neg = s[i] == '-'; i++; }
    if (i >= s.size()) return false;
    unsigned __int128 v = 0;
    for (; i < s.size(); i++) {
        if (s[i] < '0' || s[i] > '9') return false;
        v = v * 10 + (unsigned)(s[i] - '0');
        if (v > ((unsigned __int128)1 << 63)) return false;
    }
    if (!neg && v > (unsigned __int128)INT64_MAX) return false;
    *out = neg ? (int64_t)(-(__int128)v) : (int64_t)v;
    return true;
}

bool scalar_resource(const std::string& n) {
    if (n == "cpu" || n == "memory" || n == "pods" || n == "ephemeral-storage") return false;
    if (n.rfind("hugepages-", 0) == 0 || n.rfind("attachable-volumes-", 0) == 0) return true;
    if (n.find("kubernetes.io/") != std::string::npos) return true;                // IsPrefixedNativeResource
    if (n.find('/') == std::string::npos || n.rfind("requests.", 0) == 0) return false;
    return qualified_name("requests." + n);                                       // IsExtendedResourceName
}

// Toleration.ToleratesTaint (core/v1/toleration.go:38-57)
bool tolerates(const ca_toleration_str& t, const std::string& key, const std::string& value, const std::string& effect) {
    const std::string te = s_or(t.effect), tk = s_or(t.key), op = s_or(t.op), tv = s_or(t.value);
    if (!te.empty() && te != effect) return false;
    if (!tk.empty() && tk != key) return false;
    if (op.empty() || op == "Equal") return tv == value;
    return op == "Exists";
}

void set_bit(uint64_t* w, int32_t i) { w[i >> 6] |= 1ull << (i & 63); }

}  // namespace

struct ca_interner {
    Universe taints{63};                           // bit 63: "a taint past the width"
    Universe pairs{CA_LABEL_WORDS * 64};
    Universe keys{64};
    Universe int_keys{CA_MAX_INT_KEYS};
    Universe ports{CA_PORT_WORDS * 64};
    std::unordered_set<std::string> port_groups_over;     // (protocol, port) with a triple past the width
    Universe scalars{CA_MAX_SCALAR};
    Universe names{INT32_MAX};
};

extern "C" {

int ca_interner_create(ca_interner** out) {
    if (!out) return CA_EINVAL;
    *out = new ca_interner();
    return CA_OK;
}

int ca_interner_destroy(ca_interner* it) {
    if (!it) return CA_EINVAL;
    delete it;
    return CA_OK;
}

int ca_interner_size(const ca_interner* it, int32_t universe, int32_t* n, int32_t* n_overflow) {
    if (!it) return CA_EINVAL;
    const Universe* u = nullptr;
    switch (universe) {
        case CA_U_TAINTS: u = &it->taints; break;
        case CA_U_LABEL_PAIRS: u = &it->pairs; break;
        case CA_U_LABEL_KEYS: u = &it->keys; break;
        case CA_U_INT_KEYS: u = &it->int_keys; break;
        case CA_U_PORTS: u = &it->ports; break;
        case CA_U_SCALARS: u = &it->scalars; break;
        case CA_U_NAMES: u = &it->names; break;
        default: return CA_EINVAL;
    }
    if (n) *n = (int32_t)u->ids.size();
    if (n_overflow) *n_overflow = (int32_t)u->overflow.size();
    return CA_OK;
}

int ca_is_scalar_resource(const char* name) { return name && scalar_resource(name) ? 1 : 0; }

int ca_intern_taint(ca_interner* it, const char* key, const char* value, const char* effect, int32_t* id) {
    if (!it || !id) return CA_EINVAL;
    const std::string e = s_or(effect);
    if (e != "NoSchedule" && e != "NoExecute") { *id = CA_INTERN_NOT_INTERNED; return CA_OK; }   // helpers.go:78-101
    *id = it->taints.get(key3(s_or(key), s_or(value), e), true);
    return CA_OK;
}

int ca_intern_label_pair(ca_interner* it, const char* key, const char* value, int32_t* id) {
    if (!it || !id) return CA_EINVAL;
    *id = it->pairs.get(key2(s_or(key), s_or(value)), true);
    return CA_OK;
}

int ca_intern_label_key(ca_interner* it, const char* key, int32_t* id) {
    if (!it || !id) return CA_EINVAL;
    *id = it->keys.get(s_or(key), true);
    return CA_OK;
}

int ca_intern_int_key(ca_interner* it, const char* key, int32_t* id) {
    if (!it || !id) return CA_EINVAL;
    *id = it->int_keys.get(s_or(key), true);
    return CA_OK;
}

// HostPortInfo.sanitize (SF/types.go:923-931): empty IP -> 0.0.0.0, empty protocol -> TCP;
// HostPortInfo.Add ignores host ports <= 0
int ca_intern_port(ca_interner* it, const char* host_ip, const char* protocol, int32_t host_port, int32_t* id) {
    if (!it || !id) return CA_EINVAL;
    if (host_port <= 0) { *id = CA_INTERN_NOT_INTERNED; return CA_OK; }
    std::string ip = s_or(host_ip), proto = s_or(protocol);
    if (ip.empty()) ip = "0.0.0.0";
    if (proto.empty()) proto = "TCP";
    *id = it->ports.get(key3(ip, proto, std::to_string(host_port)), true);
    if (*id < 0) it->port_groups_over.insert(key2(proto, std::to_string(host_port)));
    return CA_OK;
}

int ca_intern_resource(ca_interner* it, const char* name, int32_t* id) {
    if (!it || !id || !name) return CA_EINVAL;
    if (!scalar_resource(name)) { *id = CA_INTERN_NOT_INTERNED; return CA_OK; }
    *id = it->scalars.get(name, true);
    return CA_OK;
}

int ca_intern_name(ca_interner* it, const char* name, int32_t* id) {
    if (!it || !id) return CA_EINVAL;
    *id = it->names.get(s_or(name), true);
    return CA_OK;
}

// encode_node's label and taint fields (intern.py:Interner.encode_node)
int ca_intern_encode_node(ca_interner* it, const ca_str_pair* labels, int32_t n_labels, const ca_taint_str* taints,
                          int32_t n_taints, ca_node_spec* out) {
    if (!it || !out || n_labels < 0 || n_taints < 0 || (n_labels > 0 && !labels) || (n_taints > 0 && !taints))
        return CA_EINVAL;
    uint64_t tm = 0;
    for (int32_t i = 0; i < n_taints; i++) {
        const std::string e = s_or(taints[i].effect);
        if (e != "NoSchedule" && e != "NoExecute") continue;
        const int32_t id = it->taints.get(key3(s_or(taints[i].key), s_or(taints[i].value), e), true);
        tm |= 1ull << (id < 0 ? 63 : id);
    }
    out->taints = tm;
    std::memset(out->label_pairs, 0, sizeof out->label_pairs);
    out->label_keys = 0;
    std::memset(out->int_label, 0, sizeof out->int_label);
    out->int_label_valid = 0;
    std::unordered_map<std::string, std::string> lab;
    for (int32_t i = 0; i < n_labels; i++) {
        const std::string k = s_or(labels[i].key), v = s_or(labels[i].value);
        lab[k] = v;
        const int32_t p = it->pairs.get(key2(k, v), false);
        if (p >= 0) set_bit(out->label_pairs, p);
        const int32_t q = it->keys.get(k, false);
        if (q >= 0) out->label_keys |= 1ull << q;
    }
    for (int32_t i = 0; i < (int32_t)it->int_keys.keys.size(); i++) {
        auto f = lab.find(it->int_keys.keys[i]);
        int64_t v = 0;
        if (f != lab.end() && parse_int64(f->second, &v)) {
            out->int_label[i] = v;
            out->int_label_valid |= 1u << i;
        }
    }
    return CA_OK;
}

// tolerated_taints and CA_POD_TOLERATES_UNSCHED (intern.py:_encode_pod, tolerations)
int ca_intern_encode_tolerations(const ca_interner* it, const ca_toleration_str* t, int32_t n, ca_pod_spec* out,
                                 int32_t* out_of_scope) {
    if (!it || !out || n < 0 || (n > 0 && !t)) return CA_EINVAL;
    uint64_t tol = 0;
    std::string k, v, e;
    for (int32_t id = 0; id < (int32_t)it->taints.keys.size(); id++) {
        split3(it->taints.keys[id], k, v, e);
        for (int32_t i = 0; i < n; i++)
            if (tolerates(t[i], k, v, e)) { tol |= 1ull << id; break; }
    }
    int32_t over = 0;
    if (!it->taints.overflow.empty()) {
        // bit 63 stands for every taint past the width: exact when the pod tolerates all of
        // them or none; otherwise the pod needs the reference path
        size_t n_tol = 0;
        for (const std::string& key : it->taints.overflow) {
            split3(key, k, v, e);
            for (int32_t i = 0; i < n; i++)
                if (tolerates(t[i], k, v, e)) { n_tol++; break; }
        }
        if (n_tol == it->taints.overflow.size()) tol |= 1ull << 63;
        else if (n_tol) over = 1;
    }
    out->tolerated_taints = tol;
    bool unsched = false;
    for (int32_t i = 0; i < n && !unsched; i++)
        unsched = tolerates(t[i], "node.kubernetes.io/unschedulable", "", "NoSchedule");
    if (unsched) out->flags |= CA_POD_TOLERATES_UNSCHED;
    else out->flags &= ~(uint32_t)CA_POD_TOLERATES_UNSCHED;
    if (out_of_scope) *out_of_scope = over;
    return CA_OK;
}

// port_conflict / port_use (HostPortInfo.CheckConflict, SF/types.go:887-921)
int ca_intern_encode_ports(ca_interner* it, const ca_port_str* p, int32_t n, ca_pod_spec* out, int32_t* out_of_scope) {
    if (!it || !out || n < 0 || (n > 0 && !p)) return CA_EINVAL;
    std::memset(out->port_conflict, 0, sizeof out->port_conflict);
    std::memset(out->port_use, 0, sizeof out->port_use);
    int32_t over = 0;
    std::string ip2, proto2, port2;
    for (int32_t i = 0; i < n; i++) {
        if (p[i].host_port <= 0) continue;
        std::string ip = s_or(p[i].host_ip), proto = s_or(p[i].protocol);
        if (ip.empty()) ip = "0.0.0.0";
        if (proto.empty()) proto = "TCP";
        const std::string port = std::to_string(p[i].host_port);
        const int32_t id = it->ports.get(key3(ip, proto, port), true);
        if (id < 0 || it->port_groups_over.count(key2(proto, port))) {
            over = 1;
            if (id < 0) continue;
        }
        set_bit(out->port_use, id);
        for (int32_t j = 0; j < (int32_t)it->ports.keys.size(); j++) {
            split3(it->ports.keys[j], ip2, proto2, port2);
            if (proto2 != proto || port2 != port) continue;
            if (ip == "0.0.0.0" || ip2 == "0.0.0.0" || ip2 == ip) set_bit(out->port_conflict, j);
        }
    }
    if (out_of_scope) *out_of_scope = over;
    return CA_OK;
}

// spec.nodeSelector pairs (AND)
int ca_intern_encode_node_selector(ca_interner* it, const ca_str_pair* sel, int32_t n, ca_pod_spec* out,
                                   int32_t* out_of_scope) {
    if (!it || !out || n < 0 || (n > 0 && !sel)) return CA_EINVAL;
    std::memset(out->node_selector, 0, sizeof out->node_selector);
    int32_t over = 0;
    for (int32_t i = 0; i < n; i++) {
        const int32_t id = it->pairs.get(key2(s_or(sel[i].key), s_or(sel[i].value)), true);
        if (id < 0) { over = 1; continue; }
        set_bit(out->node_selector, id);
    }
    if (out_of_scope) *out_of_scope = over;
    return CA_OK;
}

// One nodeSelectorTerm's requirement rows (intern.py:_compile_term; nodeaffinity.go:223-293,
// selector.go:223-267): match expressions, then match fields, in the caller's order; a
// term with an invalid requirement compiles to one CA_OP_FALSE row.
int ca_intern_compile_term(ca_interner* it, const ca_requirement_str* reqs, int32_t n, ca_selector_req* out,
                           int32_t cap, int32_t* n_rows, int32_t* out_of_scope) {
    if (!it || !n_rows || n < 0 || (n > 0 && !reqs) || cap < 0 || (cap > 0 && !out)) return CA_EINVAL;
    std::vector<ca_selector_req> rows;
    bool bad = false;
    int32_t over = 0;
    auto row = [](int32_t op, int32_t key, int64_t bound) {
        ca_selector_req r;
        std::memset(&r, 0, sizeof r);
        r.op = op; r.key = key; r.bound = bound;
        return r;
    };
    for (int32_t i = 0; i < n; i++) {
        const ca_requirement_str& q = reqs[i];
        const std::string key = s_or(q.key), op = s_or(q.op);
        if (q.n_values < 0 || (q.n_values > 0 && !q.values)) return CA_EINVAL;
        std::vector<std::string> vals;
        for (int32_t j = 0; j < q.n_values; j++) vals.push_back(s_or(q.values[j]));
        if (q.is_field) {                                      // nodeSelectorRequirementsAsFieldSelector
            if ((op != "In" && op != "NotIn") || vals.size() != 1) { bad = true; continue; }
            if (key == "metadata.name") {
                const int32_t nid = it->names.get(vals[0], true);
                rows.push_back(row(op == "In" ? CA_OP_FIELD_EQ : CA_OP_FIELD_NE, nid, 0));
            } else {
                // fields.Set.Get(missing) == "": In [v] matches iff v == "", NotIn iff v != ""
                const bool ok = op == "In" ? vals[0].empty() : !vals[0].empty();
                if (!ok) bad = true;
            }
            continue;
        }
        bool valid = qualified_name(key);
        for (const std::string& v : vals) valid = valid && label_value(v);
        if (!valid) { bad = true; continue; }
        if (op == "In" || op == "NotIn") {
            if (vals.empty()) { bad = true; continue; }
            ca_selector_req r = row(op == "In" ? CA_OP_IN : CA_OP_NOTIN, 0, 0);
            for (const std::string& v : vals) {
                const int32_t id = it->pairs.get(key2(key, v), true);
                if (id < 0) over = 1;
                else set_bit(r.pairs, id);
            }
            rows.push_back(r);
        } else if (op == "Exists" || op == "DoesNotExist") {
            if (!vals.empty()) { bad = true; continue; }
            const int32_t k = it->keys.get(key, true);
            if (k < 0) over = 1;
            rows.push_back(row(op == "Exists" ? CA_OP_EXISTS : CA_OP_DOESNOTEXIST, k < 0 ? 0 : k, 0));
        } else if (op == "Gt" || op == "Lt") {
            int64_t v = 0;
            if (vals.size() != 1 || !parse_int64(vals[0], &v)) { bad = true; continue; }
            const int32_t k = it->int_keys.get(key, true);
            if (k < 0) over = 1;
            rows.push_back(row(op == "Gt" ? CA_OP_GT : CA_OP_LT, k < 0 ? 0 : k, v));
        } else {
            bad = true;
        }
    }
    if (bad) rows.assign(1, row(CA_OP_FALSE, 0, 0));
    *n_rows = (int32_t)rows.size();
    if (out_of_scope) *out_of_scope = over;
    if ((int32_t)rows.size() > cap) return CA_ECAPACITY;
    for (size_t i = 0; i < rows.size(); i++) out[i] = rows[i];
    return CA_OK;
}

}  // extern "C"
