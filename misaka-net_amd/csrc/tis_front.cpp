// tis_front.cpp -- parser and lowering for TIS networks.
//
// The reference tokenises each line with ~18 anchored RE2 patterns
// (internal/tis/tokenizer.go:29-106).  Here a line is first cut into
// lexemes -- maximal runs of \w, maximal runs of \s, and single other bytes --
// and each instruction form is a short lexeme grammar.  Every pattern of the
// reference puts a non-\w element (\s, ',', ':' or end of text) after each
// word-class element, so matching whole \w-runs accepts exactly the language
// the regexes accept.  Character classes follow Go RE2: \s = [\t\n\f\r ],
// \w = [0-9A-Za-z_], \d = [0-9] (no \v, no Unicode).
#include "tis_front.h"

#include <algorithm>
#include <cstdio>
#include <cstring>

#include "../../include/mk.h"

namespace mk {

namespace {

inline bool is_space(unsigned char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\f' || c == '\r'; }
inline bool is_digit(unsigned char c) { return c >= '0' && c <= '9'; }
inline bool is_word(unsigned char c)
{
    return is_digit(c) || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || c == '_';
}

enum LexKind : uint8_t { LX_WS, LX_WORD, LX_CHAR };

struct Lexeme {
    LexKind kind;
    std::string text; // WORD text or the single CHAR byte
};

std::vector<Lexeme> lex(const std::string &s)
{
    std::vector<Lexeme> out;
    size_t i = 0, n = s.size();
    while (i < n) {
        unsigned char c = (unsigned char)s[i];
        size_t j = i + 1;
        if (is_space(c)) {
            while (j < n && is_space((unsigned char)s[j])) j++;
            out.push_back({LX_WS, std::string()});
        } else if (is_word(c)) {
            while (j < n && is_word((unsigned char)s[j])) j++;
            out.push_back({LX_WORD, s.substr(i, j - i)});
        } else {
            out.push_back({LX_CHAR, s.substr(i, 1)});
        }
        i = j;
    }
    return out;
}

std::string upper(std::string s)
{
    for (auto &c : s)
        if (c >= 'a' && c <= 'z') c = (char)(c - 'a' + 'A');
    return s;
}

// Grammar elements.
enum El : uint8_t {
    E_KW,    // WORD == keyword (given per form)
    E_WS1,   // \s+
    E_INT,   // -?\d+                  -> capture
    E_SRC,   // ACC|NIL|R[0123]        -> capture
    E_ACCNIL,// ACC|NIL                -> capture
    E_NET,   // \w+:R[0123]            -> capture
    E_NAME,  // \w+                    -> capture
    E_COMMA, // \s*,\s+
    E_END,   // \s*$
};

struct Matcher {
    const std::vector<Lexeme> &lx;
    size_t p = 0;
    std::vector<std::string> caps;

    explicit Matcher(const std::vector<Lexeme> &l) : lx(l) {}
    bool at(LexKind k) const { return p < lx.size() && lx[p].kind == k; }
    bool at_char(char c) const { return at(LX_CHAR) && lx[p].text[0] == c; }
    void skip_ws() { if (at(LX_WS)) p++; }

    bool word_in(std::initializer_list<const char *> set)
    {
        if (!at(LX_WORD)) return false;
        for (const char *w : set)
            if (lx[p].text == w) { caps.push_back(lx[p].text); p++; return true; }
        return false;
    }

    bool el(El e, const char *kw)
    {
        switch (e) {
        case E_KW:
            if (!at(LX_WORD) || lx[p].text != kw) return false;
            p++;
            return true;
        case E_WS1:
            if (!at(LX_WS)) return false;
            p++;
            return true;
        case E_INT: {
            std::string t;
            size_t q = p;
            if (at_char('-')) { t = "-"; q++; }
            if (q >= lx.size() || lx[q].kind != LX_WORD) return false;
            for (char c : lx[q].text)
                if (!is_digit((unsigned char)c)) return false;
            t += lx[q].text;
            caps.push_back(t);
            p = q + 1;
            return true;
        }
        case E_SRC: return word_in({"ACC", "NIL", "R0", "R1", "R2", "R3"});
        case E_ACCNIL: return word_in({"ACC", "NIL"});
        case E_NET: {
            if (p + 2 >= lx.size()) return false;
            if (lx[p].kind != LX_WORD || lx[p + 1].kind != LX_CHAR || lx[p + 1].text[0] != ':' ||
                lx[p + 2].kind != LX_WORD)
                return false;
            const std::string &r = lx[p + 2].text;
            if (!(r == "R0" || r == "R1" || r == "R2" || r == "R3")) return false;
            caps.push_back(lx[p].text + ":" + r);
            p += 3;
            return true;
        }
        case E_NAME:
            if (!at(LX_WORD)) return false;
            caps.push_back(lx[p].text);
            p++;
            return true;
        case E_COMMA:
            skip_ws();
            if (!at_char(',')) return false;
            p++;
            if (!at(LX_WS)) return false;
            p++;
            return true;
        case E_END:
            skip_ws();
            return p == lx.size();
        }
        return false;
    }
};

struct FormRule {
    Form form;
    const char *kw;
    El seq[8];
};

// One rule per reference branch, in tokenizer.go order (:47-99).  Keyword
// alternations of the reference (NOP|SWP|SAV|NEG, ADD|SUB, JMP|...) are
// expanded into one rule per keyword.
const FormRule kRules[] = {
    {F_NOP, "NOP", {E_KW, E_END}},
    {F_SWP, "SWP", {E_KW, E_END}},
    {F_SAV, "SAV", {E_KW, E_END}},
    {F_NEG, "NEG", {E_KW, E_END}},
    {F_MOV_VAL_LOCAL, "MOV", {E_KW, E_WS1, E_INT, E_COMMA, E_ACCNIL, E_END}},
    {F_MOV_VAL_NETWORK, "MOV", {E_KW, E_WS1, E_INT, E_COMMA, E_NET, E_END}},
    {F_MOV_SRC_LOCAL, "MOV", {E_KW, E_WS1, E_SRC, E_COMMA, E_ACCNIL, E_END}},
    {F_MOV_SRC_NETWORK, "MOV", {E_KW, E_WS1, E_SRC, E_COMMA, E_NET, E_END}},
    {F_ADD_VAL, "ADD", {E_KW, E_WS1, E_INT, E_END}},
    {F_SUB_VAL, "SUB", {E_KW, E_WS1, E_INT, E_END}},
    {F_ADD_SRC, "ADD", {E_KW, E_WS1, E_SRC, E_END}},
    {F_SUB_SRC, "SUB", {E_KW, E_WS1, E_SRC, E_END}},
    {F_JMP, "JMP", {E_KW, E_WS1, E_NAME, E_END}},
    {F_JEZ, "JEZ", {E_KW, E_WS1, E_NAME, E_END}},
    {F_JNZ, "JNZ", {E_KW, E_WS1, E_NAME, E_END}},
    {F_JGZ, "JGZ", {E_KW, E_WS1, E_NAME, E_END}},
    {F_JLZ, "JLZ", {E_KW, E_WS1, E_NAME, E_END}},
    {F_JRO_VAL, "JRO", {E_KW, E_WS1, E_INT, E_END}},
    {F_JRO_SRC, "JRO", {E_KW, E_WS1, E_SRC, E_END}},
    {F_PUSH_VAL, "PUSH", {E_KW, E_WS1, E_INT, E_COMMA, E_NAME, E_END}},
    {F_PUSH_SRC, "PUSH", {E_KW, E_WS1, E_SRC, E_COMMA, E_NAME, E_END}},
    {F_POP, "POP", {E_KW, E_WS1, E_NAME, E_COMMA, E_ACCNIL, E_END}},
    {F_IN, "IN", {E_KW, E_WS1, E_ACCNIL, E_END}},
    {F_OUT_VAL, "OUT", {E_KW, E_WS1, E_INT, E_END}},
    {F_OUT_SRC, "OUT", {E_KW, E_WS1, E_SRC, E_END}},
};

bool match_rule(const FormRule &r, const std::vector<Lexeme> &lx, std::vector<std::string> &caps)
{
    Matcher m(lx);
    for (El e : r.seq) {
        if (!m.el(e, r.kw)) return false;
        if (e == E_END) { caps = std::move(m.caps); return true; }
    }
    return false;
}

// ^\s*(\w+):  -> length of the match, 0 if none; label text in *word.
size_t label_prefix(const std::string &s, std::string *word)
{
    size_t i = 0, n = s.size();
    while (i < n && is_space((unsigned char)s[i])) i++;
    size_t w0 = i;
    while (i < n && is_word((unsigned char)s[i])) i++;
    if (i == w0 || i >= n || s[i] != ':') return 0;
    if (word) *word = s.substr(w0, i - w0);
    return i + 1;
}

std::vector<std::string> split_lines(const std::string &s)
{
    std::vector<std::string> out;
    size_t st = 0;
    for (;;) {
        size_t nl = s.find('\n', st);
        if (nl == std::string::npos) { out.push_back(s.substr(st)); break; }
        out.push_back(s.substr(st, nl - st));
        st = nl + 1;
    }
    return out;
}

} // namespace

const char *form_name(Form f)
{
    static const char *names[F_COUNT] = {
        "NOP", "SWP", "SAV", "NEG", "MOV_VAL_LOCAL", "MOV_VAL_NETWORK", "MOV_SRC_LOCAL",
        "MOV_SRC_NETWORK", "ADD_VAL", "SUB_VAL", "ADD_SRC", "SUB_SRC", "JMP", "JEZ", "JNZ", "JGZ",
        "JLZ", "JRO_VAL", "JRO_SRC", "PUSH_VAL", "PUSH_SRC", "POP", "IN", "OUT_VAL", "OUT_SRC"};
    return f < F_COUNT ? names[f] : "?";
}

int Program::label_line(const std::string &u) const
{
    for (auto &kv : labels)
        if (kv.first == u) return kv.second;
    return -1;
}

bool atoi64(const std::string &tok, int64_t &v)
{
    // tok matches -?\d+ ; strconv.Atoi accepts it unless out of int64 range.
    bool neg = !tok.empty() && tok[0] == '-';
    unsigned __int128 acc = 0;
    const unsigned __int128 lim = neg ? ((unsigned __int128)1 << 63) : (((unsigned __int128)1 << 63) - 1);
    for (size_t i = neg ? 1 : 0; i < tok.size(); i++) {
        acc = acc * 10 + (unsigned)(tok[i] - '0');
        if (acc > lim) return false;
    }
    uint64_t u = (uint64_t)acc;
    v = neg ? (int64_t)(0 - u) : (int64_t)u;
    return true;
}

bool parse_program(const std::string &src, Program &out, std::string &err)
{
    out = Program();
    std::vector<std::string> lines = split_lines(src); // program.go:179
    // GenerateLabelMap (tokenizer.go:11-26)
    for (size_t i = 0; i < lines.size(); i++) {
        std::string w;
        if (label_prefix(lines[i], &w)) {
            std::string u = upper(w);
            if (out.label_line(u) >= 0) { err = "Cannot repeat label"; return false; }
            out.labels.emplace_back(u, (int)i);
        }
    }
    // Tokenize (tokenizer.go:29-106)
    out.lines.reserve(lines.size());
    for (size_t i = 0; i < lines.size(); i++) {
        const std::string &raw = lines[i];
        size_t cut = label_prefix(raw, nullptr);
        while (cut < raw.size() && is_space((unsigned char)raw[cut])) cut++;
        std::string instr = raw.substr(cut);
        Line ln{F_NOP, "", ""};
        if (instr.empty() || instr[0] == '#') { out.lines.push_back(ln); continue; }
        std::vector<Lexeme> lx = lex(instr);
        bool ok = false;
        for (const FormRule &r : kRules) {
            std::vector<std::string> caps;
            if (!match_rule(r, lx, caps)) continue;
            ln.form = r.form;
            if (caps.size() > 0) ln.a = caps[0];
            if (caps.size() > 1) ln.b = caps[1];
            if (r.form >= F_JMP && r.form <= F_JLZ) {
                ln.a = upper(ln.a);
                if (out.label_line(ln.a) < 0) {
                    char buf[64];
                    snprintf(buf, sizeof buf, "line %zu, label '", i);
                    err = std::string(buf) + ln.a + "' was not declared";
                    return false;
                }
            }
            ok = true;
            break;
        }
        if (!ok) {
            char buf[64];
            snprintf(buf, sizeof buf, "line %zu, '", i);
            err = std::string(buf) + instr + "' not a valid instruction";
            return false;
        }
        out.lines.push_back(ln);
    }
    return true;
}

namespace {

struct Resolver {
    const Network &net;
    const std::vector<NodeSpec> &nodes;
    // returns NK_PROGRAM/NK_STACK/NK_MASTER with index, or -1 for unknown
    int find(const std::string &name, int &idx) const
    {
        for (int i = 0; i < net.nprog; i++)
            if (net.prog_names[i] == name) { idx = i; return NK_PROGRAM; }
        for (int i = 0; i < net.nstack; i++)
            if (net.stack_names[i] == name) { idx = i; return NK_STACK; }
        for (auto &n : nodes)
            if (n.kind == NK_MASTER && n.name == name) { idx = 0; return NK_MASTER; }
        for (size_t i = 0; i < net.remote_names.size(); i++)
            if (net.remote_names[i] == name) { idx = (int)i; return net.remote_kinds[i]; }
        return -1;
    }
};

uint8_t src_of(const std::string &t)
{
    if (t == "ACC") return SRC_ACC;
    if (t == "NIL") return SRC_NIL;
    return (uint8_t)(SRC_R0 + (t[1] - '0'));
}

inline bool is_port(uint8_t s) { return s >= SRC_R0; }

// A network op whose RPC can never succeed.  Unknown host: the Dial never
// returns, after the source operand was already fetched (program.go:
// 268-272 then :492).  Wrong service type: Unimplemented error, update()
// retried forever, each retry re-fetching the source (program.go:80-92).
Insn failing_network_op(int kind, uint8_t src, int64_t imm)
{
    Insn in{};
    in.src = src;
    in.imm = imm;
    if (kind < 0) in.op = OP_HANG;
    else in.op = is_port(src) ? OP_RETRY : OP_STUCK;
    return in;
}

} // namespace

int lower_network(const std::vector<NodeSpec> &nodes, Network &net, std::string &err)
{
    net = Network();
    if (nodes.size() > 4096) { err = "too many nodes"; return MK_ELIMIT; }
    std::vector<const NodeSpec *> progs, stacks;
    int nmaster = 0;
    for (size_t i = 0; i < nodes.size(); i++) {
        for (size_t j = i + 1; j < nodes.size(); j++)
            if (nodes[i].name == nodes[j].name) { err = "duplicate node name " + nodes[i].name; return MK_EINVAL; }
        switch (nodes[i].kind) {
        case NK_PROGRAM: progs.push_back(&nodes[i]); break;
        case NK_STACK: stacks.push_back(&nodes[i]); break;
        case NK_MASTER: nmaster++; break;
        case NK_REMOTE_PROGRAM: case NK_REMOTE_STACK:
            net.remote_names.push_back(nodes[i].name);
            net.remote_kinds.push_back(nodes[i].kind);
            break;
        default: err = "invalid node type"; return MK_EINVAL; // master.go:437
        }
    }
    if (nmaster > 1) { err = "more than one master node"; return MK_EINVAL; }
    if (progs.empty()) { err = "network has no program node"; return MK_EINVAL; }
    if ((int)progs.size() > MK_MAX_PROGRAM_NODES) { err = "too many program nodes (max 16)"; return MK_ELIMIT; }
    if ((int)stacks.size() > MK_MAX_STACK_NODES) { err = "too many stack nodes (max 32)"; return MK_ELIMIT; }
    auto by_name = [](const NodeSpec *a, const NodeSpec *b) { return a->name < b->name; };
    std::sort(progs.begin(), progs.end(), by_name); // canonical schedule order
    std::sort(stacks.begin(), stacks.end(), by_name);
    net.nprog = (int)progs.size();
    net.nstack = (int)stacks.size();
    for (auto *p : progs) net.prog_names.push_back(p->name);
    for (auto *s : stacks) net.stack_names.push_back(s->name);

    std::vector<Program> parsed(progs.size());
    for (size_t i = 0; i < progs.size(); i++) {
        std::string e;
        if (!parse_program(progs[i]->program, parsed[i], e)) {
            err = "node " + progs[i]->name + ": " + e;
            return MK_EPARSE;
        }
        if (parsed[i].lines.size() > MK_MAX_LINES) {
            err = "node " + progs[i]->name + ": program too long";
            return MK_ELIMIT;
        }
    }

    Resolver R{net, nodes};
    for (size_t pi = 0; pi < progs.size(); pi++) {
        const Program &P = parsed[pi];
        net.base.push_back((uint32_t)net.code.size());
        net.len.push_back((uint32_t)P.lines.size());
        for (const Line &L : P.lines) {
            Insn in{};
            in.op = OP_NOP;
            in.src = SRC_NIL;
            int64_t v = 0;
            bool imm_ok = true;
            switch (L.form) {
            case F_MOV_VAL_LOCAL: case F_MOV_VAL_NETWORK: case F_ADD_VAL: case F_SUB_VAL:
            case F_JRO_VAL: case F_PUSH_VAL: case F_OUT_VAL:
                // Atoi runs first on every execution; a range error makes the
                // instruction fail forever before any side effect.
                imm_ok = atoi64(L.a, v);
                break;
            default: break;
            }
            if (!imm_ok) { in.op = OP_STUCK; net.code.push_back(in); continue; }
            switch (L.form) {
            case F_NOP: in.op = OP_NOP; break;
            case F_SWP: in.op = OP_SWP; break;
            case F_SAV: in.op = OP_SAV; break;
            case F_NEG: in.op = OP_NEG; break;
            case F_MOV_VAL_LOCAL: in.op = OP_MOV; in.src = SRC_IMM; in.imm = v; in.dst = L.b == "ACC"; break;
            case F_MOV_SRC_LOCAL: in.op = OP_MOV; in.src = src_of(L.a); in.dst = L.b == "ACC"; break;
            case F_MOV_VAL_NETWORK: case F_MOV_SRC_NETWORK: {
                uint8_t s = L.form == F_MOV_VAL_NETWORK ? (uint8_t)SRC_IMM : src_of(L.a);
                size_t colon = L.b.find(':');
                std::string host = L.b.substr(0, colon);
                int k = L.b[colon + 2] - '0', idx = 0;
                int kind = R.find(host, idx);
                if (kind == NK_PROGRAM) {
                    in.op = OP_SEND; in.src = s; in.imm = v; in.arg = (uint16_t)(idx * 4 + k);
                } else if (kind == NK_REMOTE_PROGRAM) {
                    in.op = OP_XSEND; in.src = s; in.imm = v; in.arg = (uint16_t)(idx * 4 + k);
                    net.uses_remote = true;
                } else {
                    in = failing_network_op(kind, s, v);
                }
                break;
            }
            case F_ADD_VAL: in.op = OP_ADD; in.src = SRC_IMM; in.imm = v; break;
            case F_SUB_VAL: in.op = OP_SUB; in.src = SRC_IMM; in.imm = v; break;
            case F_ADD_SRC: in.op = OP_ADD; in.src = src_of(L.a); break;
            case F_SUB_SRC: in.op = OP_SUB; in.src = src_of(L.a); break;
            case F_JMP: case F_JEZ: case F_JNZ: case F_JGZ: case F_JLZ:
                in.op = (uint8_t)(OP_JMP + (L.form - F_JMP));
                in.arg = (uint16_t)P.label_line(L.a);
                break;
            case F_JRO_VAL: in.op = OP_JRO; in.src = SRC_IMM; in.imm = v; break;
            case F_JRO_SRC: in.op = OP_JRO; in.src = src_of(L.a); break;
            case F_PUSH_VAL: case F_PUSH_SRC: {
                uint8_t s = L.form == F_PUSH_VAL ? (uint8_t)SRC_IMM : src_of(L.a);
                int idx = 0, kind = R.find(L.b, idx);
                if (kind == NK_STACK) {
                    in.op = OP_PUSH; in.src = s; in.imm = v; in.arg = (uint16_t)idx;
                    net.uses_stacks = true;
                } else if (kind == NK_REMOTE_STACK) {
                    in.op = OP_XPUSH; in.src = s; in.imm = v; in.arg = (uint16_t)idx;
                    net.uses_remote = true;
                } else {
                    in = failing_network_op(kind, s, v);
                }
                break;
            }
            case F_POP: {
                int idx = 0, kind = R.find(L.a, idx);
                if (kind == NK_STACK) {
                    in.op = OP_POP; in.arg = (uint16_t)idx; in.dst = L.b == "ACC";
                    net.uses_stacks = true;
                } else if (kind == NK_REMOTE_STACK) {
                    in.op = OP_XPOP; in.arg = (uint16_t)idx; in.dst = L.b == "ACC";
                    net.uses_remote = true;
                } else {
                    in = failing_network_op(kind, SRC_NIL, 0);
                }
                break;
            }
            case F_IN: in.op = OP_IN; in.dst = L.a == "ACC"; break;
            case F_OUT_VAL: in.op = OP_OUT; in.src = SRC_IMM; in.imm = v; break;
            case F_OUT_SRC: in.op = OP_OUT; in.src = src_of(L.a); break;
            default: in.op = OP_STUCK; break;
            }
            net.code.push_back(in);
        }
    }
    return MK_OK;
}

std::string disasm(const Network &net)
{
    static const char *ops[OP_COUNT] = {"NOP", "SWP", "SAV", "NEG", "MOV", "ADD", "SUB",
                                        "JMP", "JEZ", "JNZ", "JGZ", "JLZ", "JRO", "SEND",
                                        "PUSH", "POP", "IN", "OUT", "STUCK", "HANG", "RETRY",
                                        "XSEND", "XPUSH", "XPOP"};
    static const char *srcs[] = {"IMM", "ACC", "NIL", "R0", "R1", "R2", "R3"};
    std::string s;
    char buf[160];
    for (int n = 0; n < net.nprog; n++) {
        s += "node " + net.prog_names[n] + "\n";
        for (uint32_t i = 0; i < net.len[n]; i++) {
            const Insn &in = net.code[net.base[n] + i];
            snprintf(buf, sizeof buf, "  %3u %-5s src=%s dst=%u arg=%u imm=%lld\n", i,
                     in.op < OP_COUNT ? ops[in.op] : "?", in.src <= SRC_R3 ? srcs[in.src] : "?",
                     in.dst, in.arg, (long long)in.imm);
            s += buf;
        }
    }
    return s;
}

} // namespace mk
