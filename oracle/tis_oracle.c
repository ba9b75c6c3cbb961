/*
 * tis_oracle.c -- CPU restatement of jasmaa/misaka-net's program/stack-node
 * execution path.  TEST INFRASTRUCTURE ONLY: this file is the parity checker.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it; the product path (misaka-net_amd/) never links or calls it.
 *
 * Pinning status (see DESIGN.md "Oracle"):
 *   The reference is Go 1.14 (go.mod:3) and cannot be built or run here (no Go
 *   toolchain; grpc-go v1.33.1 / protobuf v1.25.0 not vendored).  It ships no
 *   tests, golden vectors or fixtures.  The only in-tree known answer is
 *   README.md:39-44 (the docker-compose example network returns input + 2);
 *   this oracle is pinned against it in tests/test_oracle_kat.py.  Every other
 *   behaviour is restated from the Go source and the Go 1.14 language/stdlib
 *   semantics it relies on (two's-complement int64 wrap, int32() truncation,
 *   strconv.Atoi range rules, RE2 ASCII classes) -- parity for those is
 *   "hand-derived, otherwise unpinned".
 *
 * Structure deliberately mirrors the reference rather than the product:
 *   - programs are tokenised into string tokens exactly like tis.Tokenize
 *     (tokenizer.go:29-106), labels via tis.GenerateLabelMap (tokenizer.go:11-26);
 *   - the interpreter switches on the token string and re-parses immediates
 *     with a strconv.Atoi restatement on every execution (program.go:219-432);
 *   - network targets are resolved by name on every execution, like the
 *     per-call grpc.Dial (program.go:475-566).
 *
 * Lane model: a lane is a fresh post-/reset, post-/run
 * copy of the network with one /compute input deposited in the master's inChan.
 * Canonical schedule: rounds; in each round every program node (sorted by name,
 * byte order) attempts exactly one update(); effects are visible immediately to
 * later nodes.  A lane ends at quiescence (a round with no state change), when
 * retired instructions reach the budget at a round end, on stack overflow
 * (bounded stand-in for the reference's unbounded IntStack), or optionally at
 * the first OUT.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define ORC_MAX_NODES 64
#include "orc_flat.h"

/* status byte layout (shared with include/mk.h) */
#define ST_QUIESCENT 1
#define ST_BUDGET 2
#define ST_STACK_OVERFLOW 3
#define ST_OUTPUT_STOP 4
#define ST_CALL_OPEN 6 /* sessions: a call is still open on this instance (nothing done) */
#define ST_HAS_OUTPUT 0x10

/* ------------------------------------------------------------------------ */
/* Go RE2 ASCII classes: \s = [\t\n\f\r ], \w = [0-9A-Za-z_], \d = [0-9]     */
/* ------------------------------------------------------------------------ */
static int re_s(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\f' || c == '\r'; }
static int re_d(char c) { return c >= '0' && c <= '9'; }
static int re_w(char c)
{
    return re_d(c) || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '_';
}

/* A cursor over one line.  Every pattern used by tokenizer.go is a sequence
 * of elements whose character classes are pairwise disjoint at each boundary,
 * so a greedy left-to-right match is the unique RE2 match. */
typedef struct {
    const char *p, *e;
} cur_t;

typedef struct {
    const char *p;
    size_t n;
} cap_t;

static int c_lit(cur_t *c, const char *lit)
{
    size_t n = strlen(lit);
    if ((size_t)(c->e - c->p) < n || memcmp(c->p, lit, n) != 0)
        return 0;
    c->p += n;
    return 1;
}
static void c_sstar(cur_t *c)
{
    while (c->p < c->e && re_s(*c->p))
        c->p++;
}
static int c_splus(cur_t *c)
{
    if (c->p >= c->e || !re_s(*c->p))
        return 0;
    c_sstar(c);
    return 1;
}
static int c_end(cur_t *c) /* \s*$ */
{
    c_sstar(c);
    return c->p == c->e;
}
static int c_word(cur_t *c, cap_t *cap) /* (\w+) */
{
    const char *s = c->p;
    while (c->p < c->e && re_w(*c->p))
        c->p++;
    if (c->p == s)
        return 0;
    cap->p = s;
    cap->n = (size_t)(c->p - s);
    return 1;
}
static int c_int(cur_t *c, cap_t *cap) /* (-?\d+) */
{
    const char *s = c->p;
    if (c->p < c->e && *c->p == '-')
        c->p++;
    const char *d = c->p;
    while (c->p < c->e && re_d(*c->p))
        c->p++;
    if (c->p == d) {
        c->p = s;
        return 0;
    }
    cap->p = s;
    cap->n = (size_t)(c->p - s);
    return 1;
}
static int c_alt(cur_t *c, const char *const *alts, cap_t *cap) /* (A|B|...) */
{
    for (int i = 0; alts[i]; i++) {
        cur_t t = *c;
        if (c_lit(&t, alts[i])) {
            cap->p = c->p;
            cap->n = strlen(alts[i]);
            *c = t;
            return 1;
        }
    }
    return 0;
}
static const char *const A_ACCNIL[] = {"ACC", "NIL", NULL};
static const char *const A_SRC[] = {"ACC", "NIL", "R0", "R1", "R2", "R3", NULL};
static const char *const A_NSSN[] = {"NOP", "SWP", "SAV", "NEG", NULL};
static const char *const A_ADDSUB[] = {"ADD", "SUB", NULL};
static const char *const A_JMP[] = {"JMP", "JEZ", "JNZ", "JGZ", "JLZ", NULL};
static const char *const A_REG[] = {"R0", "R1", "R2", "R3", NULL};

static int c_netreg(cur_t *c, cap_t *cap) /* (\w+:R[0123]) */
{
    cur_t t = *c;
    cap_t w, r;
    if (!c_word(&t, &w) || !c_lit(&t, ":") || !c_alt(&t, A_REG, &r))
        return 0;
    cap->p = c->p;
    cap->n = (size_t)(t.p - c->p);
    *c = t;
    return 1;
}
static int c_comma(cur_t *c) /* \s*,\s+ */
{
    c_sstar(c);
    if (!c_lit(c, ","))
        return 0;
    return c_splus(c);
}

/* ------------------------------------------------------------------------ */
/* strconv.Atoi restatement (Go 1.14, 64-bit int): [+-]?[0-9]+, range check */
/* ------------------------------------------------------------------------ */
/* returns 0 ok, 1 syntax error, 2 range error */
int orc_go_atoi(const char *s, size_t n, int64_t *out)
{
    size_t i = 0;
    int neg = 0;
    if (n == 0)
        return 1;
    if (s[0] == '+' || s[0] == '-') {
        neg = s[0] == '-';
        i = 1;
        if (n == 1)
            return 1;
    }
    uint64_t v = 0;
    const uint64_t lim = neg ? (uint64_t)1 << 63 : ((uint64_t)1 << 63) - 1;
    int range = 0;
    for (; i < n; i++) {
        if (!re_d(s[i]))
            return 1;
        uint64_t d = (uint64_t)(s[i] - '0');
        if (!range) {
            if (v > (lim - d) / 10)
                range = 1;
            else
                v = v * 10 + d;
        }
    }
    if (range)
        return 2;
    *out = neg ? (int64_t)(0 - v) : (int64_t)v;
    return 0;
}

/* ------------------------------------------------------------------------ */
/* Programs: [][]string tokens + label map, as tis.Tokenize produces them    */
/* ------------------------------------------------------------------------ */
typedef struct {
    int ntok;
    char *tok[3];
} orc_ins;

typedef struct {
    int n;
    orc_ins *ins;
    int nlab;
    char **lab;
    int *labidx;
} orc_prog;

static char *xstrndup(const char *p, size_t n)
{
    char *s = (char *)malloc(n + 1);
    memcpy(s, p, n);
    s[n] = 0;
    return s;
}

static void prog_free(orc_prog *pg)
{
    if (!pg)
        return;
    for (int i = 0; i < pg->n; i++)
        for (int t = 0; t < pg->ins[i].ntok; t++)
            free(pg->ins[i].tok[t]);
    free(pg->ins);
    for (int i = 0; i < pg->nlab; i++)
        free(pg->lab[i]);
    free(pg->lab);
    free(pg->labidx);
    memset(pg, 0, sizeof *pg);
}

static int lab_find(const orc_prog *pg, const char *name)
{
    for (int i = 0; i < pg->nlab; i++)
        if (strcmp(pg->lab[i], name) == 0)
            return pg->labidx[i];
    return -1;
}

static void upcase(char *s)
{
    for (; *s; s++)
        if (*s >= 'a' && *s <= 'z')
            *s = (char)(*s - 'a' + 'A');
}

static void set_tok(orc_ins *in, int ntok, const char *a, size_t an, const char *b, size_t bn,
                    const char *c, size_t cn)
{
    in->ntok = ntok;
    in->tok[0] = xstrndup(a, an);
    if (ntok > 1)
        in->tok[1] = xstrndup(b, bn);
    if (ntok > 2)
        in->tok[2] = xstrndup(c, cn);
}

/* Split lines exactly like strings.Split(s, "\n") (program.go:179). */
typedef struct {
    int n;
    const char **p;
    size_t *len;
} lines_t;

static void split_lines(const char *s, lines_t *L)
{
    size_t total = strlen(s);
    int n = 1;
    for (size_t i = 0; i < total; i++)
        n += s[i] == '\n';
    L->n = n;
    L->p = (const char **)malloc(sizeof(char *) * (size_t)n);
    L->len = (size_t *)malloc(sizeof(size_t) * (size_t)n);
    const char *st = s;
    int k = 0;
    for (size_t i = 0; i <= total; i++) {
        if (i == total || s[i] == '\n') {
            L->p[k] = st;
            L->len[k] = (size_t)(s + i - st);
            k++;
            st = s + i + 1;
        }
    }
}

/* tis.GenerateLabelMap (tokenizer.go:11-26) + tis.Tokenize (tokenizer.go:29-106).
 * Returns 0 on success, -1 with the Go error text in err. */
static int orc_load_program(const char *src, orc_prog *pg, char *err, size_t errlen)
{
    lines_t L;
    memset(pg, 0, sizeof *pg);
    split_lines(src, &L);
    pg->lab = (char **)calloc((size_t)L.n, sizeof(char *));
    pg->labidx = (int *)calloc((size_t)L.n, sizeof(int));
    /* GenerateLabelMap: ^\s*(\w+): */
    for (int i = 0; i < L.n; i++) {
        cur_t c = {L.p[i], L.p[i] + L.len[i]};
        cap_t w;
        c_sstar(&c);
        if (c_word(&c, &w) && c_lit(&c, ":")) {
            char *lab = xstrndup(w.p, w.n);
            upcase(lab);
            if (lab_find(pg, lab) >= 0) {
                free(lab);
                snprintf(err, errlen, "Cannot repeat label");
                goto fail;
            }
            pg->lab[pg->nlab] = lab;
            pg->labidx[pg->nlab] = i;
            pg->nlab++;
        }
    }
    pg->n = L.n;
    pg->ins = (orc_ins *)calloc((size_t)L.n, sizeof(orc_ins));
    for (int i = 0; i < L.n; i++) {
        cur_t c = {L.p[i], L.p[i] + L.len[i]};
        orc_ins *in = &pg->ins[i];
        /* prefix ^(\s*\w+:)?\s* */
        {
            cur_t t = c;
            cap_t w;
            c_sstar(&t);
            if (c_word(&t, &w) && c_lit(&t, ":"))
                c = t;
            c_sstar(&c);
        }
        const cur_t s0 = c;
        cap_t a, b, m;
        if (c.p == c.e) {
            set_tok(in, 1, "NOP", 3, 0, 0, 0, 0);
            continue;
        }
        if (*c.p == '#') { /* ^#.*$ (no '\n' can remain after the split) */
            set_tok(in, 1, "NOP", 3, 0, 0, 0, 0);
            continue;
        }
        c = s0;
        if (c_alt(&c, A_NSSN, &m) && c_end(&c)) {
            set_tok(in, 1, m.p, m.n, 0, 0, 0, 0);
            continue;
        }
        c = s0;
        if (c_lit(&c, "MOV") && c_splus(&c) && c_int(&c, &a) && c_comma(&c) &&
            c_alt(&c, A_ACCNIL, &b) && c_end(&c)) {
            set_tok(in, 3, "MOV_VAL_LOCAL", 13, a.p, a.n, b.p, b.n);
            continue;
        }
        c = s0;
        if (c_lit(&c, "MOV") && c_splus(&c) && c_int(&c, &a) && c_comma(&c) && c_netreg(&c, &b) &&
            c_end(&c)) {
            set_tok(in, 3, "MOV_VAL_NETWORK", 15, a.p, a.n, b.p, b.n);
            continue;
        }
        c = s0;
        if (c_lit(&c, "MOV") && c_splus(&c) && c_alt(&c, A_SRC, &a) && c_comma(&c) &&
            c_alt(&c, A_ACCNIL, &b) && c_end(&c)) {
            set_tok(in, 3, "MOV_SRC_LOCAL", 13, a.p, a.n, b.p, b.n);
            continue;
        }
        c = s0;
        if (c_lit(&c, "MOV") && c_splus(&c) && c_alt(&c, A_SRC, &a) && c_comma(&c) &&
            c_netreg(&c, &b) && c_end(&c)) {
            set_tok(in, 3, "MOV_SRC_NETWORK", 15, a.p, a.n, b.p, b.n);
            continue;
        }
        c = s0;
        if (c_alt(&c, A_ADDSUB, &m) && c_splus(&c) && c_int(&c, &a) && c_end(&c)) {
            char op[8];
            snprintf(op, sizeof op, "%.3s_VAL", m.p);
            set_tok(in, 2, op, 7, a.p, a.n, 0, 0);
            continue;
        }
        c = s0;
        if (c_alt(&c, A_ADDSUB, &m) && c_splus(&c) && c_alt(&c, A_SRC, &a) && c_end(&c)) {
            char op[8];
            snprintf(op, sizeof op, "%.3s_SRC", m.p);
            set_tok(in, 2, op, 7, a.p, a.n, 0, 0);
            continue;
        }
        c = s0;
        if (c_alt(&c, A_JMP, &m) && c_splus(&c) && c_word(&c, &a) && c_end(&c)) {
            char *lab = xstrndup(a.p, a.n);
            upcase(lab);
            if (lab_find(pg, lab) < 0) {
                snprintf(err, errlen, "line %d, label '%s' was not declared", i, lab);
                free(lab);
                goto fail;
            }
            set_tok(in, 2, m.p, m.n, lab, strlen(lab), 0, 0);
            free(lab);
            continue;
        }
        c = s0;
        if (c_lit(&c, "JRO") && c_splus(&c) && c_int(&c, &a) && c_end(&c)) {
            set_tok(in, 2, "JRO_VAL", 7, a.p, a.n, 0, 0);
            continue;
        }
        c = s0;
        if (c_lit(&c, "JRO") && c_splus(&c) && c_alt(&c, A_SRC, &a) && c_end(&c)) {
            set_tok(in, 2, "JRO_SRC", 7, a.p, a.n, 0, 0);
            continue;
        }
        c = s0;
        if (c_lit(&c, "PUSH") && c_splus(&c) && c_int(&c, &a) && c_comma(&c) && c_word(&c, &b) &&
            c_end(&c)) {
            set_tok(in, 3, "PUSH_VAL", 8, a.p, a.n, b.p, b.n);
            continue;
        }
        c = s0;
        if (c_lit(&c, "PUSH") && c_splus(&c) && c_alt(&c, A_SRC, &a) && c_comma(&c) &&
            c_word(&c, &b) && c_end(&c)) {
            set_tok(in, 3, "PUSH_SRC", 8, a.p, a.n, b.p, b.n);
            continue;
        }
        c = s0;
        if (c_lit(&c, "POP") && c_splus(&c) && c_word(&c, &a) && c_comma(&c) &&
            c_alt(&c, A_ACCNIL, &b) && c_end(&c)) {
            set_tok(in, 3, "POP", 3, a.p, a.n, b.p, b.n);
            continue;
        }
        c = s0;
        if (c_lit(&c, "IN") && c_splus(&c) && c_alt(&c, A_ACCNIL, &a) && c_end(&c)) {
            set_tok(in, 2, "IN", 2, a.p, a.n, 0, 0);
            continue;
        }
        c = s0;
        if (c_lit(&c, "OUT") && c_splus(&c) && c_int(&c, &a) && c_end(&c)) {
            set_tok(in, 2, "OUT_VAL", 7, a.p, a.n, 0, 0);
            continue;
        }
        c = s0;
        if (c_lit(&c, "OUT") && c_splus(&c) && c_alt(&c, A_SRC, &a) && c_end(&c)) {
            set_tok(in, 2, "OUT_SRC", 7, a.p, a.n, 0, 0);
            continue;
        }
        snprintf(err, errlen, "line %d, '%.*s' not a valid instruction", i, (int)(s0.e - s0.p), s0.p);
        goto fail;
    }
    free(L.p);
    free(L.len);
    return 0;
fail:
    free(L.p);
    free(L.len);
    prog_free(pg);
    return -1;
}

/* Test hook: tokenise one program.  On success writes lines separated by
 * '\n', tokens separated by '\x1f', returns 0.  On error writes the Go error
 * text, returns -1.  Output is truncated to outlen. */
int orc_tokenize(const char *src, char *out, size_t outlen)
{
    orc_prog pg;
    char err[4096];
    if (orc_load_program(src, &pg, err, sizeof err) != 0) {
        snprintf(out, outlen, "%s", err);
        return -1;
    }
    size_t o = 0;
    out[0] = 0;
    for (int i = 0; i < pg.n; i++) {
        for (int t = 0; t < pg.ins[i].ntok; t++) {
            int w = snprintf(out + o, o < outlen ? outlen - o : 0, "%s%s", t ? "\x1f" : "",
                             pg.ins[i].tok[t]);
            o += (size_t)w;
        }
        if (i + 1 < pg.n) {
            int w = snprintf(out + o, o < outlen ? outlen - o : 0, "\n");
            o += (size_t)w;
        }
    }
    prog_free(&pg);
    return o < outlen ? 0 : -2;
}

/* Test hook: label map as "LABEL=idx\n" lines in insertion order. */
int orc_label_map(const char *src, char *out, size_t outlen)
{
    orc_prog pg;
    char err[4096];
    if (orc_load_program(src, &pg, err, sizeof err) != 0) {
        snprintf(out, outlen, "%s", err);
        return -1;
    }
    size_t o = 0;
    out[0] = 0;
    for (int i = 0; i < pg.nlab; i++) {
        int w = snprintf(out + o, o < outlen ? outlen - o : 0, "%s=%d\n", pg.lab[i], pg.labidx[i]);
        o += (size_t)w;
    }
    prog_free(&pg);
    return o < outlen ? 0 : -2;
}

/* ------------------------------------------------------------------------ */
/* Network                                                                   */
/* ------------------------------------------------------------------------ */
enum { K_PROGRAM = 0, K_STACK = 1 };
enum { T_UNKNOWN = 0, T_PROGRAM, T_STACK, T_MASTER };

typedef struct {
    int nprog, nstack;
    char *pname[ORC_MAX_NODES]; /* program nodes, sorted by name */
    orc_prog prog[ORC_MAX_NODES];
    char *sname[ORC_MAX_NODES]; /* stack nodes, sorted by name */
    char *master;               /* may be NULL */
} orc_net;

static int cmpstr(const void *a, const void *b)
{
    return strcmp(*(char *const *)a, *(char *const *)b);
}

void orc_net_free(orc_net *net)
{
    if (!net)
        return;
    for (int i = 0; i < net->nprog; i++) {
        free(net->pname[i]);
        prog_free(&net->prog[i]);
    }
    for (int i = 0; i < net->nstack; i++)
        free(net->sname[i]);
    free(net->master);
    free(net);
}

/* kinds: 0 = program, 1 = stack.  Program nodes whose text fails to load
 * report "node <name>: <go error>" (first failing node in sorted order). */
orc_net *orc_net_load(int n, const char *const *names, const int *kinds, const char *const *programs,
                      const char *master, char *err, size_t errlen)
{
    if (n <= 0 || n > ORC_MAX_NODES) {
        snprintf(err, errlen, "invalid node count");
        return NULL;
    }
    for (int i = 0; i < n; i++)
        for (int j = i + 1; j < n; j++)
            if (strcmp(names[i], names[j]) == 0) {
                snprintf(err, errlen, "duplicate node name %s", names[i]);
                return NULL;
            }
    orc_net *net = (orc_net *)calloc(1, sizeof(orc_net));
    int order[ORC_MAX_NODES];
    const char *sorted[ORC_MAX_NODES];
    for (int i = 0; i < n; i++)
        sorted[i] = names[i];
    qsort(sorted, (size_t)n, sizeof(char *), cmpstr);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++)
            if (names[j] == sorted[i] || strcmp(names[j], sorted[i]) == 0) {
                order[i] = j;
                break;
            }
    for (int i = 0; i < n; i++) {
        int j = order[i];
        if (kinds[j] == K_PROGRAM) {
            char e2[4096];
            int k = net->nprog;
            if (orc_load_program(programs[j] ? programs[j] : "", &net->prog[k], e2, sizeof e2) != 0) {
                snprintf(err, errlen, "node %s: %s", names[j], e2);
                orc_net_free(net);
                return NULL;
            }
            net->pname[k] = xstrndup(names[j], strlen(names[j]));
            net->nprog++;
        } else if (kinds[j] == K_STACK) {
            net->sname[net->nstack++] = xstrndup(names[j], strlen(names[j]));
        } else {
            snprintf(err, errlen, "invalid node type");
            orc_net_free(net);
            return NULL;
        }
    }
    if (master)
        net->master = xstrndup(master, strlen(master));
    return net;
}

static int resolve(const orc_net *net, const char *name, size_t len, int *idx)
{
    for (int i = 0; i < net->nprog; i++)
        if (strlen(net->pname[i]) == len && memcmp(net->pname[i], name, len) == 0) {
            *idx = i;
            return T_PROGRAM;
        }
    for (int i = 0; i < net->nstack; i++)
        if (strlen(net->sname[i]) == len && memcmp(net->sname[i], name, len) == 0) {
            *idx = i;
            return T_STACK;
        }
    if (net->master && strlen(net->master) == len && memcmp(net->master, name, len) == 0)
        return T_MASTER;
    return T_UNKNOWN;
}

/* ------------------------------------------------------------------------ */
/* Lane state                                                                */
/* ------------------------------------------------------------------------ */
typedef struct {
    int64_t acc, bak; /* Go int (program.go:27-28) */
    int ptr;
    int full[4];      /* r0..r3: chan int, cap 1 (program.go:29-32, bufferSize :21) */
    int64_t val[4];
    int pend;         /* blocked inside Send/SendOutput with value pendval */
    int64_t pendval;
    int hung;         /* goroutine stuck forever in grpc.Dial(WithBlock) to an unknown host */
} pnode_t;

typedef struct {
    int64_t *v;
    uint32_t n;
} stk_t;

typedef struct {
    pnode_t node[ORC_MAX_NODES];
    stk_t stk[ORC_MAX_NODES];
    int in_avail;
    int64_t in_val;
    int out_cnt;
    int64_t out_val;
    uint32_t steps;
    uint32_t stack_cap;
    /* stateful sessions (row f2): outChan is a capacity-1 channel emptied by
     * each /compute, instead of the single-/compute out_cnt rule */
    int session;
    int out_full;
    uint8_t dead; /* reason the session ended (0 = alive): a stack overflow */
    /* the open /compute call: its input (deposited into inChan or not yet),
     * and the instructions it has retired over its earlier slices */
    int call_open, call_dep;
    int64_t call_x;
    uint32_t call_steps;
    /* a call imported mid-slice (orc_session_import): instructions its
     * slice has already retired, and where the round stands */
    uint32_t slice_carry;
    int res_pos, res_changed;
} lane_t;

enum { R_NONE = 0, R_CHANGED = 1, R_RETIRED = 3, R_OVERFLOW = 4 };

/* getFromSrc (program.go:434-472).  Returns 1 when a value was obtained,
 * 0 when the receive would block.  *consumed is set for R0..R3. */
static int get_src(pnode_t *nd, const char *src, int64_t *v, int *consumed)
{
    if (strcmp(src, "ACC") == 0) {
        *v = nd->acc;
        return 1;
    }
    if (strcmp(src, "NIL") == 0) {
        *v = 0;
        return 1;
    }
    if (src[0] == 'R') {
        int k = src[1] - '0';
        if (!nd->full[k])
            return 0;
        *v = nd->val[k];
        nd->full[k] = 0;
        *consumed = 1;
        return 1;
    }
    return 0; /* unreachable: tokenizer restricts sources */
}

static void advance(pnode_t *nd, const orc_prog *pg, lane_t *ln)
{
    nd->ptr = (nd->ptr + 1) % pg->n; /* program.go:429 */
    ln->steps++;
}

/* sendValue (program.go:475-506) + Program.Send (program.go:160-175). */
static int net_send(const orc_net *net, lane_t *ln, pnode_t *nd, int64_t v, const char *target,
                    int consumed)
{
    const char *colon = strchr(target, ':');
    int k = colon[2] - '0', m;
    int t = resolve(net, target, (size_t)(colon - target), &m);
    if (t == T_UNKNOWN) { /* grpc.Dial WithBlock never returns (program.go:72,492) */
        nd->hung = 1;
        return R_CHANGED;
    }
    if (t != T_PROGRAM) /* Unimplemented RPC -> error -> retried (program.go:80-92) */
        return consumed ? R_CHANGED : R_NONE;
    pnode_t *dst = &ln->node[m];
    if (dst->full[k]) { /* p.rK <- v blocks while full */
        if (nd->pend)
            return R_NONE;
        nd->pend = 1;
        nd->pendval = v;
        return R_CHANGED;
    }
    dst->full[k] = 1;
    dst->val[k] = (int64_t)(int32_t)v; /* SendMessage{Value: int32(v)} (program.go:498) */
    nd->pend = 0;
    return R_RETIRED;
}

/* outputValue (program.go:554-566) + Master.SendOutput (master.go:245-249). */
static int net_out(lane_t *ln, pnode_t *nd, int64_t v)
{
    if (ln->session) { /* outChan <- v blocks while full (master.go:246, cap 1 :59) */
        if (ln->out_full) {
            if (nd->pend)
                return R_NONE;
            nd->pend = 1;
            nd->pendval = v;
            return R_CHANGED;
        }
        ln->out_full = 1;
        ln->out_val = (int64_t)(int32_t)v;
        nd->pend = 0;
        return R_RETIRED;
    }
    if (ln->out_cnt >= 2) { /* outChan (cap 1) full and /compute reads only once */
        if (nd->pend)
            return R_NONE;
        nd->pend = 1;
        nd->pendval = v;
        return R_CHANGED;
    }
    if (ln->out_cnt == 0)
        ln->out_val = (int64_t)(int32_t)v; /* ValueMessage{Value: int32(v)} (program.go:561) */
    ln->out_cnt++;
    nd->pend = 0;
    return R_RETIRED;
}

/* pushValue (program.go:509-521) + Stack.Push (stack.go:95-105). */
static int net_push(const orc_net *net, lane_t *ln, pnode_t *nd, int64_t v, const char *target,
                    int consumed)
{
    int m;
    int t = resolve(net, target, strlen(target), &m);
    if (t == T_UNKNOWN) {
        nd->hung = 1;
        return R_CHANGED;
    }
    if (t != T_STACK)
        return consumed ? R_CHANGED : R_NONE;
    stk_t *s = &ln->stk[m];
    if (s->n >= ln->stack_cap)
        return R_OVERFLOW;
    s->v[s->n++] = (int64_t)(int32_t)v; /* ValueMessage{Value: int32(v)} (program.go:516) */
    return R_RETIRED;
}

/* One update() of program node n (program.go:219-432) under the lane model. */
static int attempt(const orc_net *net, lane_t *ln, int n)
{
    pnode_t *nd = &ln->node[n];
    const orc_prog *pg = &net->prog[n];
    if (nd->hung)
        return R_NONE;
    const orc_ins *in = &pg->ins[nd->ptr];
    const char *op = in->tok[0];
    int64_t v = 0;
    int consumed = 0, r;

    if (strcmp(op, "NOP") == 0) {
    } else if (strcmp(op, "MOV_VAL_LOCAL") == 0) {
        if (orc_go_atoi(in->tok[1], strlen(in->tok[1]), &v))
            return R_NONE; /* Atoi error: retried forever */
        if (strcmp(in->tok[2], "ACC") == 0)
            nd->acc = v;
    } else if (strcmp(op, "MOV_VAL_NETWORK") == 0) {
        if (nd->pend)
            v = nd->pendval;
        else if (orc_go_atoi(in->tok[1], strlen(in->tok[1]), &v))
            return R_NONE;
        r = net_send(net, ln, nd, v, in->tok[2], 0);
        if (r != R_RETIRED)
            return r;
    } else if (strcmp(op, "MOV_SRC_LOCAL") == 0) {
        if (!get_src(nd, in->tok[1], &v, &consumed))
            return R_NONE;
        if (strcmp(in->tok[2], "ACC") == 0)
            nd->acc = v;
    } else if (strcmp(op, "MOV_SRC_NETWORK") == 0) {
        if (nd->pend)
            v = nd->pendval;
        else if (!get_src(nd, in->tok[1], &v, &consumed))
            return R_NONE;
        r = net_send(net, ln, nd, v, in->tok[2], consumed);
        if (r != R_RETIRED)
            return r;
    } else if (strcmp(op, "SWP") == 0) {
        int64_t t = nd->acc;
        nd->acc = nd->bak;
        nd->bak = t;
    } else if (strcmp(op, "SAV") == 0) {
        nd->bak = nd->acc;
    } else if (strcmp(op, "ADD_VAL") == 0 || strcmp(op, "SUB_VAL") == 0) {
        if (orc_go_atoi(in->tok[1], strlen(in->tok[1]), &v))
            return R_NONE;
        if (op[0] == 'A')
            nd->acc = (int64_t)((uint64_t)nd->acc + (uint64_t)v);
        else
            nd->acc = (int64_t)((uint64_t)nd->acc - (uint64_t)v);
    } else if (strcmp(op, "ADD_SRC") == 0 || strcmp(op, "SUB_SRC") == 0) {
        if (!get_src(nd, in->tok[1], &v, &consumed))
            return R_NONE;
        if (op[0] == 'A')
            nd->acc = (int64_t)((uint64_t)nd->acc + (uint64_t)v);
        else
            nd->acc = (int64_t)((uint64_t)nd->acc - (uint64_t)v);
    } else if (strcmp(op, "NEG") == 0) {
        nd->acc = (int64_t)(0 - (uint64_t)nd->acc);
    } else if (strcmp(op, "JMP") == 0 || strcmp(op, "JEZ") == 0 || strcmp(op, "JNZ") == 0 ||
               strcmp(op, "JGZ") == 0 || strcmp(op, "JLZ") == 0) {
        int take = op[1] == 'M' || (op[1] == 'E' && nd->acc == 0) ||
                   (op[1] == 'N' && nd->acc != 0) || (op[1] == 'G' && nd->acc > 0) ||
                   (op[1] == 'L' && nd->acc < 0);
        if (take) {
            nd->ptr = lab_find(pg, in->tok[1]);
            ln->steps++;
            return R_RETIRED;
        }
    } else if (strcmp(op, "JRO_VAL") == 0 || strcmp(op, "JRO_SRC") == 0) {
        if (op[4] == 'V') {
            if (orc_go_atoi(in->tok[1], strlen(in->tok[1]), &v))
                return R_NONE;
        } else if (!get_src(nd, in->tok[1], &v, &consumed)) {
            return R_NONE;
        }
        /* utils.IntClamp(p.ptr+v, 0, len(p.asm)-1) with int64 wrap (math.go:20-22) */
        int64_t t = (int64_t)((uint64_t)(int64_t)nd->ptr + (uint64_t)v);
        int64_t hi = pg->n - 1;
        if (t > hi)
            t = hi;
        if (t < 0)
            t = 0;
        nd->ptr = (int)t;
        ln->steps++;
        return R_RETIRED;
    } else if (strcmp(op, "PUSH_VAL") == 0 || strcmp(op, "PUSH_SRC") == 0) {
        if (op[5] == 'V') {
            if (orc_go_atoi(in->tok[1], strlen(in->tok[1]), &v))
                return R_NONE;
        } else if (!get_src(nd, in->tok[1], &v, &consumed)) {
            return R_NONE;
        }
        r = net_push(net, ln, nd, v, in->tok[2], consumed);
        if (r != R_RETIRED)
            return r;
    } else if (strcmp(op, "POP") == 0) {
        int m;
        int t = resolve(net, in->tok[1], strlen(in->tok[1]), &m);
        if (t == T_UNKNOWN) {
            nd->hung = 1;
            return R_CHANGED;
        }
        if (t != T_STACK)
            return R_NONE;
        stk_t *s = &ln->stk[m];
        if (s->n == 0) /* waitPop blocks (stack.go:133-155) */
            return R_NONE;
        v = s->v[--s->n];
        if (strcmp(in->tok[2], "ACC") == 0)
            nd->acc = v;
    } else if (strcmp(op, "IN") == 0) {
        if (!ln->in_avail) /* <-m.inChan blocks (master.go:233-242) */
            return R_NONE;
        ln->in_avail = 0;
        v = (int64_t)(int32_t)ln->in_val; /* ValueMessage{Value: int32(v)} (master.go:237) */
        if (strcmp(in->tok[1], "ACC") == 0)
            nd->acc = v;
    } else if (strcmp(op, "OUT_VAL") == 0 || strcmp(op, "OUT_SRC") == 0) {
        if (nd->pend)
            v = nd->pendval;
        else if (op[4] == 'V') {
            if (orc_go_atoi(in->tok[1], strlen(in->tok[1]), &v))
                return R_NONE;
        } else if (!get_src(nd, in->tok[1], &v, &consumed)) {
            return R_NONE;
        }
        r = net_out(ln, nd, v);
        if (r != R_RETIRED)
            return r;
    } else {
        return R_NONE; /* default: "not a valid instruction" (unreachable) */
    }
    advance(nd, pg, ln);
    return R_RETIRED;
}

typedef struct {
    uint32_t budget;
    uint32_t stack_cap;
    int stop_on_output;
} orc_opts;

static void lane_reset(const orc_net *net, lane_t *ln, int64_t input)
{
    for (int i = 0; i < net->nprog; i++)
        memset(&ln->node[i], 0, sizeof(pnode_t));
    for (int i = 0; i < net->nstack; i++)
        ln->stk[i].n = 0;
    ln->in_avail = 1;
    ln->in_val = input;
    ln->out_cnt = 0;
    ln->out_val = 0;
    ln->steps = 0;
}

static uint8_t run_lane(const orc_net *net, lane_t *ln, int64_t input, const orc_opts *o)
{
    lane_reset(net, ln, input);
    for (;;) {
        int changed = 0;
        for (int n = 0; n < net->nprog; n++) {
            int r = attempt(net, ln, n);
            if (r & R_OVERFLOW)
                return ST_STACK_OVERFLOW;
            changed |= r & R_CHANGED;
            if (o->stop_on_output && ln->out_cnt > 0)
                return ST_OUTPUT_STOP;
        }
        if (!changed)
            return ST_QUIESCENT;
        if (ln->steps >= o->budget)
            return ST_BUDGET;
    }
}

/* Lane trace (the reference's per-instruction
 * log.Printf, program.go:222-223, as data): run_lane for one input,
 * recording every retired instruction -- round, program node (sorted-name
 * index), the ptr it executed at, ACC and BAK after it -- up to `max`
 * entries.  Returns the lane status; *count = entries written. */
typedef struct {
    uint32_t round;
    uint16_t node;
    uint16_t ip;
    int64_t acc;
    int64_t bak;
} orc_trace_entry;

static lane_t *lane_alloc(const orc_net *net, uint32_t cap);
static void lane_free(const orc_net *net, lane_t *ln);

int orc_trace_lane(const orc_net *net, int64_t input, uint32_t budget, uint32_t stack_cap, int stop_on_output,
                   orc_trace_entry *out, uint32_t max, uint32_t *count)
{
    lane_t *ln = lane_alloc(net, stack_cap);
    lane_reset(net, ln, input);
    uint32_t k = 0, round = 0;
    uint8_t st;
    for (;;) {
        int changed = 0, over = 0, stop = 0;
        for (int n = 0; n < net->nprog; n++) {
            const int ip = ln->node[n].ptr;
            int r = attempt(net, ln, n);
            if (r == R_RETIRED && k < max) {
                out[k].round = round;
                out[k].node = (uint16_t)n;
                out[k].ip = (uint16_t)ip;
                out[k].acc = ln->node[n].acc;
                out[k].bak = ln->node[n].bak;
                k++;
            }
            if (r & R_OVERFLOW) {
                over = 1;
                break;
            }
            changed |= r & R_CHANGED;
            if (stop_on_output && ln->out_cnt > 0) {
                stop = 1;
                break;
            }
        }
        if (over) { st = ST_STACK_OVERFLOW; break; }
        if (stop) { st = ST_OUTPUT_STOP; break; }
        if (!changed) { st = ST_QUIESCENT; break; }
        if (ln->steps >= budget) { st = ST_BUDGET; break; }
        round++;
    }
    if (ln->out_cnt > 0)
        st |= ST_HAS_OUTPUT;
    *count = k;
    lane_free(net, ln);
    return st;
}

static lane_t *lane_alloc(const orc_net *net, uint32_t cap)
{
    lane_t *ln = (lane_t *)calloc(1, sizeof(lane_t));
    ln->stack_cap = cap;
    for (int i = 0; i < net->nstack; i++)
        ln->stk[i].v = (int64_t *)malloc(sizeof(int64_t) * (cap ? cap : 1));
    return ln;
}

static void lane_free_n(int nstack, lane_t *ln)
{
    for (int i = 0; i < nstack; i++)
        free(ln->stk[i].v);
    free(ln);
}

static void lane_free(const orc_net *net, lane_t *ln) { lane_free_n(net->nstack, ln); }

typedef struct {
    const orc_net *net;
    const int64_t *in;
    int32_t *out;
    uint8_t *status;
    uint32_t *steps;
    size_t lo, hi;
    orc_opts o;
} job_t;

static void *worker(void *arg)
{
    job_t *j = (job_t *)arg;
    lane_t *ln = lane_alloc(j->net, j->o.stack_cap);
    for (size_t i = j->lo; i < j->hi; i++) {
        uint8_t st = run_lane(j->net, ln, j->in[i], &j->o);
        if (ln->out_cnt > 0)
            st |= ST_HAS_OUTPUT;
        j->out[i] = (int32_t)ln->out_val;
        j->status[i] = st;
        if (j->steps)
            j->steps[i] = ln->steps;
    }
    lane_free(j->net, ln);
    return NULL;
}

/* Evaluate n independent /compute inputs.  in[] holds strconv.Atoi values
 * (int64); they are truncated to int32 at GetInput exactly like master.go:237. */
int orc_compute_batch(const orc_net *net, const int64_t *in, size_t n, int32_t *out, uint8_t *status,
                      uint32_t *steps, uint32_t budget, uint32_t stack_cap, int stop_on_output,
                      int threads)
{
    if (!net || budget == 0)
        return -1;
    if (threads < 1)
        threads = 1;
    if ((size_t)threads > n)
        threads = n ? (int)n : 1;
    job_t jobs[256];
    pthread_t tid[256];
    if (threads > 256)
        threads = 256;
    orc_opts o = {budget, stack_cap, stop_on_output};
    for (int t = 0; t < threads; t++) {
        jobs[t] = (job_t){net, in, out, status, steps, n * (size_t)t / (size_t)threads,
                          n * (size_t)(t + 1) / (size_t)threads, o};
    }
    if (threads == 1) {
        worker(&jobs[0]);
        return 0;
    }
    for (int t = 0; t < threads; t++)
        pthread_create(&tid[t], NULL, worker, &jobs[t]);
    for (int t = 0; t < threads; t++)
        pthread_join(tid[t], NULL);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* Stateful sessions                            */
/* ------------------------------------------------------------------------ */
/* The reference's nodes keep running between /compute calls
 * (program.go:80-92): ACC, BAK, ptr, ports, stacks and the master's inChan /
 * outChan (capacity 1 each, master.go:58-59) persist from one call to the
 * next.  A session is one network instance under the canonical schedule; one
 * /compute call (master.go:216-219) on it:
 *   loop:
 *     if inChan is empty and the input is not deposited yet: deposit it
 *       (m.inChan <- v blocks while inChan is full, :216);
 *     if it is deposited and outChan holds a value: take it -> the result
 *       (<-m.outChan, :219), the call closes;
 *     if this slice of the call retired `budget` instructions: the slice
 *       ends with ST_BUDGET and the call stays OPEN -- the reference's
 *       handler is still waiting while its nodes run on (program.go:80-92),
 *       so session_step(resume) continues it with a fresh slice;
 *     run one round; a round without change closes the call with
 *       ST_QUIESCENT (nothing can ever change without another input: the
 *       reference's handler would block forever; here the call is abandoned
 *       and the instance stays alive for the next input, an input not yet
 *       deposited is dropped); a stack overflow (our stack_cap; the
 *       reference's stacks are unbounded) ends the session until reset.
 * A new call while one is open does nothing and reports ST_CALL_OPEN; the
 * host resumes the open call or cancels it (orc_sessions_cancel). */
typedef struct {
    const orc_net *net;
    size_t n;
    int nstack; /* freeing never touches net (a garbage collector may free it first) */
    lane_t **lanes;
} orc_sessions;

static void lane_reset_session(const orc_net *net, lane_t *ln)
{
    lane_reset(net, ln, 0);
    ln->in_avail = 0; /* inChan empty */
    ln->session = 1;
    ln->out_full = 0;
    ln->dead = 0;
    ln->call_open = ln->call_dep = 0;
    ln->call_x = 0;
    ln->call_steps = 0;
    ln->slice_carry = 0;
    ln->res_pos = ln->res_changed = 0;
}

/* One slice of a /compute call: a new call with input *x, or (x == NULL)
 * the open call resumed.  *steps = instructions the call retired so far. */
static uint8_t session_step(const orc_net *net, lane_t *ln, const int64_t *x, uint32_t budget, int32_t *out,
                            uint32_t *steps)
{
    *out = 0;
    *steps = 0;
    if (ln->dead)
        return ln->dead;
    if (!x) {
        if (!ln->call_open)
            return 0; /* nothing to resume */
    } else {
        if (ln->call_open)
            return ST_CALL_OPEN;
        ln->call_open = 1;
        ln->call_dep = 0;
        ln->call_x = *x;
        ln->call_steps = 0;
    }
    const uint32_t s0 = ln->steps, carry = ln->slice_carry;
    ln->slice_carry = 0;
    uint8_t st;
    for (;;) {
        /* an imported call may stand inside a round: finish that round first */
        const int n0 = ln->res_pos;
        int changed = ln->res_changed, over = 0;
        ln->res_pos = ln->res_changed = 0;
        if (n0 == 0) {
            if (!ln->call_dep && !ln->in_avail) {
                ln->in_avail = 1;
                ln->in_val = ln->call_x;
                ln->call_dep = 1;
            }
            if (ln->call_dep && ln->out_full) {
                ln->out_full = 0;
                *out = (int32_t)ln->out_val;
                st = ST_HAS_OUTPUT;
                ln->call_open = 0;
                break;
            }
            if (ln->steps - s0 + carry >= budget) {
                st = ST_BUDGET; /* the call stays open */
                break;
            }
        }
        for (int n = n0; n < net->nprog; n++) {
            int r = attempt(net, ln, n);
            if (r & R_OVERFLOW) {
                over = 1;
                break;
            }
            changed |= r & R_CHANGED;
        }
        if (over) {
            st = ln->dead = ST_STACK_OVERFLOW;
            ln->call_open = 0;
            break;
        }
        if (!changed) {
            st = ST_QUIESCENT;
            ln->call_open = 0;
            break;
        }
    }
    ln->call_steps += ln->steps - s0;
    *steps = ln->call_steps;
    return st;
}

orc_sessions *orc_sessions_new(const orc_net *net, size_t n, uint32_t stack_cap)
{
    orc_sessions *S = (orc_sessions *)calloc(1, sizeof(orc_sessions));
    S->net = net;
    S->n = n;
    S->nstack = net->nstack;
    S->lanes = (lane_t **)calloc(n ? n : 1, sizeof(lane_t *));
    for (size_t i = 0; i < n; i++) {
        S->lanes[i] = lane_alloc(net, stack_cap);
        lane_reset_session(net, S->lanes[i]);
    }
    return S;
}

void orc_sessions_free(orc_sessions *S)
{
    if (!S)
        return;
    for (size_t i = 0; i < S->n; i++)
        lane_free_n(S->nstack, S->lanes[i]);
    free(S->lanes);
    free(S);
}

void orc_sessions_reset(orc_sessions *S)
{
    for (size_t i = 0; i < S->n; i++)
        lane_reset_session(S->net, S->lanes[i]);
}

typedef struct {
    orc_sessions *S;
    const int64_t *in; /* NULL: resume the open calls */
    int32_t *out;
    uint8_t *status;
    uint32_t *steps;
    uint32_t budget;
    size_t lo, hi;
} sjob_t;

static void *sworker(void *arg)
{
    sjob_t *j = (sjob_t *)arg;
    for (size_t i = j->lo; i < j->hi; i++) {
        uint32_t sp;
        j->status[i] = session_step(j->S->net, j->S->lanes[i], j->in ? &j->in[i] : NULL, j->budget, &j->out[i], &sp);
        if (j->steps)
            j->steps[i] = sp;
    }
    return NULL;
}

/* One /compute call on every session i with input in[i], or (in == NULL)
 * one more slice of every open call. */
int orc_sessions_compute(orc_sessions *S, const int64_t *in, int32_t *out, uint8_t *status, uint32_t *steps,
                         uint32_t budget, int threads)
{
    if (!S || budget == 0)
        return -1;
    const size_t n = S->n;
    if (threads < 1)
        threads = 1;
    if ((size_t)threads > n)
        threads = n ? (int)n : 1;
    if (threads > 256)
        threads = 256;
    sjob_t jobs[256];
    pthread_t tid[256];
    for (int t = 0; t < threads; t++)
        jobs[t] = (sjob_t){S, in, out, status, steps, budget, n * (size_t)t / (size_t)threads,
                           n * (size_t)(t + 1) / (size_t)threads};
    if (threads == 1) {
        sworker(&jobs[0]);
        return 0;
    }
    for (int t = 0; t < threads; t++)
        pthread_create(&tid[t], NULL, sworker, &jobs[t]);
    for (int t = 0; t < threads; t++)
        pthread_join(tid[t], NULL);
    return 0;
}

/* A session's state in the interpreter's terms (mk_exec.hip's session
 * arrays for one instance), with an open call: the native tier hands a call
 * off at a superblock entry (sess_convert.h); the test infrastructure
 * imports that state here and lets the oracle finish the call. */
int orc_session_import(orc_sessions *S, size_t i, const orc_flat *f)
{
    if (!S || i >= S->n || !f) return -1;
    lane_t *ln = S->lanes[i];
    const orc_net *net = S->net;
    for (int n = 0; n < net->nprog; n++) {
        pnode_t *nd = &ln->node[n];
        nd->acc = f->acc[n];
        nd->bak = f->bak[n];
        nd->ptr = f->ip[n];
        for (int k = 0; k < 4; k++) {
            nd->full[k] = (int)((f->pfull >> (4 * n + k)) & 1u);
            nd->val[k] = f->port[4 * n + k];
        }
        nd->pend = (int)((f->pend >> n) & 1u);
        nd->pendval = f->pendv[n];
        nd->hung = (int)((f->hung >> n) & 1u);
    }
    for (int s = 0; s < net->nstack; s++) {
        if (f->depth[s] > ln->stack_cap) return -1;
        ln->stk[s].n = f->depth[s];
        for (uint32_t d = 0; d < f->depth[s]; d++) ln->stk[s].v[d] = f->entries[(size_t)s * ln->stack_cap + d];
    }
    ln->in_avail = f->in_full;
    ln->in_val = f->in_val;
    ln->out_full = f->out_full;
    ln->out_val = f->out_val;
    ln->dead = 0;
    ln->call_open = 1;
    ln->call_dep = f->deposited;
    ln->call_x = f->pin;
    ln->call_steps = f->csteps;
    ln->slice_carry = f->csteps;
    ln->res_pos = f->pos;
    ln->res_changed = f->changed;
    return 0;
}

/* Abandon every open call (the master answered it 504): its input stays
 * where it is if deposited, an undeposited one is dropped. */
void orc_sessions_cancel(orc_sessions *S)
{
    for (size_t i = 0; i < S->n; i++)
        S->lanes[i]->call_open = 0;
}

int orc_net_nprog(const orc_net *net) { return net->nprog; }
int orc_net_nstack(const orc_net *net) { return net->nstack; }

/* ------------------------------------------------------------------------ */
/* Synthetic inputs: x_i = (int32) splitmix64(seed ^ i) */
/* kind 0: full int32 range, every 16th lane (i % 16 == 15) an edge value    */
/* kind 1: splitmix64(seed ^ i) & mask                                       */
/* ------------------------------------------------------------------------ */
static uint64_t splitmix64(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static const int32_t EDGES[8] = {INT32_MIN, INT32_MIN + 1, INT32_MIN + 2, -1,
                                 0,         1,             INT32_MAX - 1, INT32_MAX};

int32_t orc_gen_one(uint64_t seed, int kind, uint32_t mask, uint64_t i)
{
    uint64_t h = splitmix64(seed ^ i);
    if (kind == 1)
        return (int32_t)(uint32_t)(h & mask);
    if ((i & 15) == 15)
        return EDGES[(h >> 32) & 7];
    return (int32_t)(uint32_t)h;
}

void orc_gen_inputs(uint64_t seed, int kind, uint32_t mask, uint64_t offset, size_t n, int64_t *out)
{
    for (size_t i = 0; i < n; i++)
        out[i] = orc_gen_one(seed, kind, mask, offset + i);
}
