/* intern_driver.c — the library's interning (casim.h "interning") from a compiled caller,
 * checked against tests/golden/intern_calls.txt: the calls a shim makes for every case of
 * tests/golden/intern_fixtures.json, with the ids and encoded fields those fixtures pin
 * (format: tests/golden/make_intern_calls.py).  Host-only: no device is touched.
 * Usage: intern_driver <intern_calls.txt>; prints "intern_driver ok <n> calls". */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "casim.h"

#define MAXTOK 4096
#define MAXSTR 512

static char* tok[MAXTOK];
static int ntok, pos;
static char strs[MAXTOK][MAXSTR];
static int nstr;
static int line_no, failures;

static const char* next(void) { return pos < ntok ? tok[pos++] : ""; }
static long long next_i(void) { return strtoll(next(), NULL, 10); }
static unsigned long long next_u(void) { return strtoull(next(), NULL, 10); }

/* hex (UTF-8) -> string; "-" -> "" */
static const char* next_s(void) {
    const char* h = next();
    char* s = strs[nstr++ % MAXTOK];
    size_t n = 0;
    if (strcmp(h, "-") != 0)
        for (size_t i = 0; h[i] && h[i + 1] && n + 1 < MAXSTR; i += 2) {
            unsigned v;
            sscanf(h + i, "%2x", &v);
            s[n++] = (char)v;
        }
    s[n] = 0;
    return s;
}

static void expect_bar(void) {
    if (strcmp(next(), "|") != 0) { fprintf(stderr, "line %d: malformed\n", line_no); exit(2); }
}

static void check_u(const char* what, unsigned long long got, unsigned long long want) {
    if (got != want) {
        fprintf(stderr, "line %d: %s = %llu, want %llu\n", line_no, what, got, want);
        failures++;
    }
}

static void check_i(const char* what, long long got, long long want) {
    if (got != want) {
        fprintf(stderr, "line %d: %s = %lld, want %lld\n", line_no, what, got, want);
        failures++;
    }
}

#define OK(x) do { int _r = (x); if (_r != CA_OK) { fprintf(stderr, "line %d: %s -> %d\n", line_no, #x, _r); exit(1); } } while (0)

int main(int argc, char** argv) {
    if (argc < 2) { fprintf(stderr, "usage: intern_driver <intern_calls.txt>\n"); return 2; }
    FILE* f = fopen(argv[1], "r");
    if (!f) { perror(argv[1]); return 2; }
    static char line[1 << 16];
    ca_interner* it = NULL;
    int calls = 0;
    while (fgets(line, sizeof line, f)) {
        line_no++;
        ntok = pos = 0;
        for (char* t = strtok(line, " \t\r\n"); t && ntok < MAXTOK; t = strtok(NULL, " \t\r\n")) tok[ntok++] = t;
        if (ntok == 0 || tok[0][0] == '#') continue;
        const char* kind = next();
        if (!strcmp(kind, "case")) {
            if (it) OK(ca_interner_destroy(it));
            OK(ca_interner_create(&it));
            continue;
        }
        calls++;
        if (!strcmp(kind, "id")) {
            const char* u = next();
            int32_t id = -99;
            if (!strcmp(u, "taint")) {
                const char* k = next_s(); const char* v = next_s(); const char* e = next_s();
                OK(ca_intern_taint(it, k, v, e, &id));
            } else if (!strcmp(u, "pair")) {
                const char* k = next_s(); const char* v = next_s();
                OK(ca_intern_label_pair(it, k, v, &id));
            } else if (!strcmp(u, "key")) {
                OK(ca_intern_label_key(it, next_s(), &id));
            } else if (!strcmp(u, "intkey")) {
                OK(ca_intern_int_key(it, next_s(), &id));
            } else if (!strcmp(u, "port")) {
                const char* ip = next_s(); const char* pr = next_s(); const int32_t pt = (int32_t)next_i();
                OK(ca_intern_port(it, ip, pr, pt, &id));
            } else if (!strcmp(u, "res")) {
                OK(ca_intern_resource(it, next_s(), &id));
            } else if (!strcmp(u, "name")) {
                OK(ca_intern_name(it, next_s(), &id));
            } else {
                fprintf(stderr, "line %d: unknown universe %s\n", line_no, u);
                return 2;
            }
            expect_bar();
            check_i(u, id, next_i());
        } else if (!strcmp(kind, "node")) {
            ca_str_pair lab[64];
            ca_taint_str tt[64];
            const int nl = (int)next_i();
            for (int i = 0; i < nl; i++) { lab[i].key = next_s(); lab[i].value = next_s(); }
            const int nt = (int)next_i();
            for (int i = 0; i < nt; i++) { tt[i].key = next_s(); tt[i].value = next_s(); tt[i].effect = next_s(); }
            ca_node_spec rec;
            memset(&rec, 0, sizeof rec);
            OK(ca_intern_encode_node(it, lab, nl, tt, nt, &rec));
            expect_bar();
            check_u("taints", rec.taints, next_u());
            for (int w = 0; w < CA_LABEL_WORDS; w++) check_u("label_pairs", rec.label_pairs[w], next_u());
            check_u("label_keys", rec.label_keys, next_u());
            for (int k = 0; k < CA_MAX_INT_KEYS; k++) check_i("int_label", rec.int_label[k], next_i());
            check_u("int_label_valid", rec.int_label_valid, next_u());
        } else if (!strcmp(kind, "tol")) {
            ca_toleration_str t[64];
            const int n = (int)next_i();
            for (int i = 0; i < n; i++) { t[i].key = next_s(); t[i].op = next_s(); t[i].value = next_s(); t[i].effect = next_s(); }
            ca_pod_spec rec;
            memset(&rec, 0, sizeof rec);
            int32_t over = 0;
            OK(ca_intern_encode_tolerations(it, t, n, &rec, &over));
            expect_bar();
            check_u("tolerated_taints", rec.tolerated_taints, next_u());
            check_i("tolerates_unsched", (rec.flags & CA_POD_TOLERATES_UNSCHED) ? 1 : 0, next_i());
        } else if (!strcmp(kind, "ports")) {
            ca_port_str p[64];
            const int n = (int)next_i();
            for (int i = 0; i < n; i++) { p[i].host_ip = next_s(); p[i].protocol = next_s(); p[i].host_port = (int32_t)next_i(); p[i].reserved = 0; }
            ca_pod_spec rec;
            memset(&rec, 0, sizeof rec);
            int32_t over = 0;
            OK(ca_intern_encode_ports(it, p, n, &rec, &over));
            expect_bar();
            for (int w = 0; w < CA_PORT_WORDS; w++) check_u("port_conflict", rec.port_conflict[w], next_u());
            for (int w = 0; w < CA_PORT_WORDS; w++) check_u("port_use", rec.port_use[w], next_u());
        } else if (!strcmp(kind, "sel")) {
            ca_str_pair s[64];
            const int n = (int)next_i();
            for (int i = 0; i < n; i++) { s[i].key = next_s(); s[i].value = next_s(); }
            ca_pod_spec rec;
            memset(&rec, 0, sizeof rec);
            int32_t over = 0;
            OK(ca_intern_encode_node_selector(it, s, n, &rec, &over));
            expect_bar();
            for (int w = 0; w < CA_LABEL_WORDS; w++) check_u("node_selector", rec.node_selector[w], next_u());
        } else if (!strcmp(kind, "term")) {
            ca_requirement_str r[64];
            const char* vals[64][16];
            const int n = (int)next_i();
            for (int i = 0; i < n; i++) {
                r[i].key = next_s(); r[i].op = next_s(); r[i].is_field = (int32_t)next_i(); r[i].n_values = (int32_t)next_i();
                for (int j = 0; j < r[i].n_values; j++) vals[i][j] = next_s();
                r[i].values = vals[i];
            }
            ca_selector_req rows[64];
            int32_t nr = 0, over = 0;
            OK(ca_intern_compile_term(it, r, n, rows, 64, &nr, &over));
            expect_bar();
            const long long want_n = next_i();
            check_i("n_rows", nr, want_n);
            for (int k = 0; k < nr && k < want_n; k++) {
                check_i("op", rows[k].op, next_i());
                check_i("key", rows[k].key, next_i());
                check_i("bound", rows[k].bound, next_i());
                for (int w = 0; w < CA_LABEL_WORDS; w++) check_u("pairs", rows[k].pairs[w], next_u());
            }
        } else {
            fprintf(stderr, "line %d: unknown call %s\n", line_no, kind);
            return 2;
        }
    }
    fclose(f);
    if (it) OK(ca_interner_destroy(it));
    if (failures) { fprintf(stderr, "intern_driver: %d mismatches\n", failures); return 1; }
    printf("intern_driver ok %d calls\n", calls);
    return 0;
}
