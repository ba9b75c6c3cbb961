// tis_front.h -- TIS program front-end: parse (internal/tis restatement) and
// lower a whole network to the executor's bytecode + wiring table.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace mk {

// Lowered opcodes.  Every reference token form (tokenizer.go:47-99) lowers to
// one of these after name resolution; forms whose execution can never
// complete lower to STUCK / HANG / RETRY (see lower_network()).
enum Op : uint8_t {
    OP_NOP = 0,
    OP_SWP,
    OP_SAV,
    OP_NEG,
    OP_MOV,   // src -> ACC|NIL                         MOV_*_LOCAL
    OP_ADD,   // ACC += src                              ADD_VAL/ADD_SRC
    OP_SUB,   // ACC -= src                              SUB_VAL/SUB_SRC
    OP_JMP,   // ip = arg                                JMP
    OP_JEZ,
    OP_JNZ,
    OP_JGZ,
    OP_JLZ,
    OP_JRO,   // ip = clamp(ip + src, 0, len-1)          JRO_VAL/JRO_SRC
    OP_SEND,  // port[arg] <- int32(src), blocks while full   MOV_*_NETWORK
    OP_PUSH,  // stack[arg].push(int32(src))             PUSH_VAL/PUSH_SRC
    OP_POP,   // ACC|NIL <- stack[arg].pop(), blocks while empty
    OP_IN,    // ACC|NIL <- int32(input), once per lane
    OP_OUT,   // output int32(src), at most 2 complete per lane
    OP_STUCK, // never completes, no side effect (Atoi range error; RPC to a wrong service without a consumed source)
    OP_HANG,  // acquire src, then hang forever (grpc.Dial WithBlock to an unknown host)
    OP_RETRY, // acquire src (consumes Rk), never retires (Unimplemented RPC retried forever)
    // Network ops to peers outside this executor (MK_NODE_REMOTE_*, row f4):
    // a stateful session hands them to the host, which makes the RPC
    // (Program.Send / Stack.Push / Stack.Pop); batch lanes have no peers and
    // block on them.
    OP_XSEND, // remote port[arg] <- int32(src) (arg = remote * 4 + k)   MOV_*_NETWORK
    OP_XPUSH, // remote stack[arg].push(int32(src))                      PUSH_*
    OP_XPOP,  // ACC|NIL <- remote stack[arg].pop()                      POP
    OP_COUNT
};

enum Src : uint8_t { SRC_IMM = 0, SRC_ACC, SRC_NIL, SRC_R0, SRC_R1, SRC_R2, SRC_R3 };

// 16-byte instruction record, read by the kernel with one scalar load.
struct Insn {
    uint8_t op;
    uint8_t src;
    uint8_t dst;  // 1 = ACC, 0 = NIL
    uint8_t rsv0;
    uint16_t arg; // jump line | port slot (node*4 + k) | stack index
    uint16_t rsv1;
    int64_t imm;
};
static_assert(sizeof(Insn) == 16, "Insn must be 16 bytes");

// Reference token forms (the asm[i][0] strings of tokenizer.go).
enum Form : uint8_t {
    F_NOP = 0, F_SWP, F_SAV, F_NEG,
    F_MOV_VAL_LOCAL, F_MOV_VAL_NETWORK, F_MOV_SRC_LOCAL, F_MOV_SRC_NETWORK,
    F_ADD_VAL, F_SUB_VAL, F_ADD_SRC, F_SUB_SRC,
    F_JMP, F_JEZ, F_JNZ, F_JGZ, F_JLZ,
    F_JRO_VAL, F_JRO_SRC,
    F_PUSH_VAL, F_PUSH_SRC, F_POP, F_IN, F_OUT_VAL, F_OUT_SRC,
    F_COUNT
};

const char *form_name(Form f);

struct Line {
    Form form;
    std::string a, b; // operand token text exactly as the reference keeps it
};

struct Program {
    std::vector<Line> lines;
    std::vector<std::pair<std::string, int>> labels; // upper-cased label -> line
    int label_line(const std::string &upper) const;
};

// Parse like ProgramNode.LoadProgram (program.go:178-193).  Returns false and
// the Go error text on failure.
bool parse_program(const std::string &src, Program &out, std::string &err);

// strconv.Atoi on a `-?\d+` token (64-bit int).  false on range error.
bool atoi64(const std::string &tok, int64_t &v);

enum NodeKind { NK_PROGRAM = 0, NK_STACK = 1, NK_MASTER = 2, NK_REMOTE_PROGRAM = 3, NK_REMOTE_STACK = 4 };

struct NodeSpec {
    std::string name;
    int kind;
    std::string program;
};

// A lowered network: program nodes sorted by name (the canonical schedule
// order), stacks sorted by name, one flat bytecode array.
struct Network {
    int nprog = 0, nstack = 0;
    std::vector<std::string> prog_names, stack_names;
    std::vector<Insn> code;
    std::vector<uint32_t> base, len; // per program node
    bool uses_stacks = false;
    // peers served elsewhere (MK_NODE_REMOTE_*), in declaration order; the
    // X-ops' remote index is into this list
    std::vector<std::string> remote_names;
    std::vector<int> remote_kinds; // NK_REMOTE_PROGRAM / NK_REMOTE_STACK
    bool uses_remote = false;
};

// Returns 0 or an MK_E* code with err filled.
int lower_network(const std::vector<NodeSpec> &nodes, Network &net, std::string &err);

std::string disasm(const Network &net);

} // namespace mk
