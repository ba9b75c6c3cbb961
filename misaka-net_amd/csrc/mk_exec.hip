// mk_exec.hip -- CDNA4 (gfx950) batched executor for TIS networks + C ABI.
//
// One lane (work-item) evaluates one /compute input through a private copy
// of the whole network (SURVEY.md section 8.0 lane model):
//   * ACC/BAK (int64), the instruction pointer and the pending-send value of
//     every program node live in VGPRs (the node loop is unrolled over the
//     template bound NMAX, so every per-node array index is static);
//   * port (R0..R3) values live in LDS rows [node*4+k][lane] -- any per-lane
//     slot index is bank-conflict free because each lane owns one column --
//     and their full bits in one 64-bit VGPR pair;
//   * stacks keep their top W entries in an LDS ring per lane and spill older
//     entries to HBM in a lane-major layout (coalesced when the lanes of a
//     wave sit at the same depth);
//   * the bytecode is read with wave-uniform (scalar) loads: for every node
//     the wave "waterfalls" over the distinct instruction pointers present
//     among its lanes, so the IP-uniform case (every lane at the same IP) is
//     one iteration with a scalar decode, and divergent lanes (JEZ/JNZ/JGZ/
//     JLZ/JRO on data) are handled group by group with ballots;
//   * a lane that finishes (quiescent / budget / overflow / output-stop)
//     writes its result and immediately takes the next input index
//     (grid-stride refill), so data-dependent trip counts do not idle lanes.
//
// Semantics restated from internal/nodes/program.go:219-566,
// internal/nodes/stack.go:95-155, internal/nodes/master.go:233-249 and
// internal/utils/math.go:20-22; see tis_front.cpp for the lowering.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <dlfcn.h>
#include <execinfo.h>
#include <fcntl.h>
#include <pthread.h>
#include <ucontext.h>
#include <sys/syscall.h>
#include <signal.h>
#include <glob.h>
#include <unistd.h>

#include <cerrno>
#include <climits>
#include <cstdint>
#include <fstream>
#include <iterator>
#include <string_view>

extern char **environ;

#include <algorithm>
#include <array>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mk.h"
#include "tis_front.h"
#include "tis_jit.h"
#include "tis_sched.h"
#define MK_HD __host__ __device__
#include "sess_convert.h"

namespace mk {

constexpr int kBlock = 256;
// The session interpreter's grid cap (blocks of kBlock, grid-stride beyond):
// 8 blocks per CU of the 256, more than its register state lets reside.
constexpr uint64_t kSessGridCap = 2048;
// Native sessions' markers (tis_jit.cpp MK_SS_*; 0xFFFFFFF0 = ended): held by
// the interpreter, handed off in this launch.
constexpr uint32_t kSessDead = 0xFFFFFFF0u, kSessT1 = 0xFFFFFFF1u, kSessHand = 0xFFFFFFF2u;
constexpr int kMaxDevices = 64;

struct KParams {
    uint32_t base[MK_MAX_PROGRAM_NODES];
    uint32_t len[MK_MAX_PROGRAM_NODES];
    int nprog;
    int nstack;
    int in_kind;
    uint32_t gen_kind;
    const void *in_data;
    uint64_t seed;
    uint64_t offset;
    uint32_t gen_mask;
    uint32_t budget;
    uint64_t n;
    int32_t *out;
    uint8_t *status;
    uint32_t *steps;
    unsigned long long *partials; // [waves][8] per-wave counters, or null
    uint32_t stack_cap;
    uint32_t flags;
    uint32_t ring;       // LDS ring entries per stack (power of two), 0 = no stacks
    uint32_t spill_rows; // stack_cap - ring (HBM entries per stack per lane)
    int32_t *spill;      // [nstack][spill_rows][lanes]
    uint64_t lanes;      // resident lanes (grid threads)
    mk_trace_entry *trace; // lane trace of input 0 (mk_trace_lane), or null
    uint32_t trace_max;
    uint32_t *trace_n;   // entries written (device)
};


#define MK_DEVICE_SRC(...) __VA_ARGS__
#include "mk_device_common.inc"
#undef MK_DEVICE_SRC

__device__ __forceinline__ int32_t lane_input(const KParams &p, uint64_t i)
{
    if (p.in_kind == MK_IN_I64) return (int32_t)((const int64_t *)p.in_data)[i]; // int32(v), master.go:237
    if (p.in_kind == MK_IN_I32) return ((const int32_t *)p.in_data)[i];
    return gen_value(p.seed, p.gen_kind, p.gen_mask, p.offset + i);
}


// Folds the per-wave partial rows into the caller's counters and clears
// them: one thread per row, a block tree in LDS, then one atomic per counter
// per block.  Rows accumulate across launches until folded (deferred stats).
__global__ void __launch_bounds__(256) stats_reduce(unsigned long long *__restrict__ partials, uint32_t nwaves,
                                                    unsigned long long *stats)
{
    __shared__ unsigned long long acc[8][256];
    const uint32_t t = threadIdx.x, w = blockIdx.x * 256 + t;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        acc[k][t] = w < nwaves ? partials[(size_t)w * 8 + k] : 0ull;
        if (w < nwaves) partials[(size_t)w * 8 + k] = 0ull;
    }
    __syncthreads();
    for (uint32_t h = 128; h > 0; h >>= 1) {
        if (t < h) {
#pragma unroll
            for (int k = 0; k < 8; k++) acc[k][t] += acc[k][t + h];
        }
        __syncthreads();
    }
    if (t < 8 && acc[t][0]) atomicAdd(&stats[t], acc[t][0]);
}


// Fetch one 16-byte instruction with a wave-uniform address as four dwords,
// so it is a single scalar load (SMEM has no byte loads) and every decoded
// field stays in SGPRs: the opcode switch is then a scalar branch.
__device__ __forceinline__ Insn fetch(const Insn *__restrict__ code, uint32_t i)
{
    const uint4 w = reinterpret_cast<const uint4 *>(code)[i];
    Insn I;
    I.op = (uint8_t)(w.x & 0xffu);
    I.src = (uint8_t)((w.x >> 8) & 0xffu);
    I.dst = (uint8_t)((w.x >> 16) & 0xffu);
    I.rsv0 = 0;
    I.arg = (uint16_t)(w.y & 0xffffu);
    I.rsv1 = 0;
    I.imm = (int64_t)(((uint64_t)w.w << 32) | (uint64_t)w.z);
    return I;
}

template <int NMAX>
__global__ void __launch_bounds__(kBlock) tis_exec(const Insn *__restrict__ code, KParams p)
{
    extern __shared__ int32_t lds[];
    const int B = kBlock;
    const int tid = threadIdx.x;
    const uint64_t gid = (uint64_t)blockIdx.x * B + tid;
    int32_t *const port = lds;                       // [nprog*4][B]
    int32_t *const sdepth = lds + p.nprog * 4 * B;   // [nstack][B]
    int32_t *const ring = sdepth + p.nstack * B;     // [nstack][W][B]
    const uint32_t W = p.ring;

    int64_t acc[NMAX], bak[NMAX];
    int32_t ip[NMAX], pendv[NMAX];
    uint32_t pend = 0, hung = 0;
    uint64_t pfull = 0;
    bool in_avail = false;
    int32_t in_val = 0, out_val = 0;
    int out_cnt = 0;
    uint32_t steps = 0;

    unsigned long long s_steps = 0, s_out = 0, s_done = 0, s_q = 0, s_b = 0, s_ov = 0, s_os = 0;

    uint64_t idx = gid;
    bool active = idx < p.n;
    uint32_t round = 0, ntrace = 0; // lane trace: rounds of input 0 and entries written

    auto init = [&](uint64_t i) {
#pragma unroll
        for (int n = 0; n < NMAX; ++n) {
            acc[n] = 0; bak[n] = 0; ip[n] = 0; pendv[n] = 0;
        }
        pend = 0; hung = 0; pfull = 0;
        in_avail = true;
        in_val = lane_input(p, i);
        out_cnt = 0; out_val = 0; steps = 0;
        for (int s = 0; s < p.nstack; ++s) sdepth[s * B + tid] = 0;
    };
    if (active) init(idx);

    while (__ballot(active) != 0ull) {
        bool changed = false, done = false;
        uint32_t reason = 0;
#pragma unroll
        for (int n = 0; n < NMAX; ++n) {
            if (n >= p.nprog) continue; // wave-uniform; keeps the loop fully unrollable
            const uint32_t len = p.len[n];
            const bool pending = active && !done && !((hung >> n) & 1u);
            if (!__ballot(pending)) continue;
            // Every lane fetches its own instruction (a 16-byte vector load of
            // hot, cache-resident code) and the op bodies below are masked
            // regions: lanes at different instructions run in ONE pass, a
            // region costs only when some lane needs it.  (The scalar-fetch
            // waterfall this replaces made one serial pass per distinct ip.)
            const int u = ip[n];
            uint4 w = make_uint4(0u, 0u, 0u, 0u);
            if (pending) w = reinterpret_cast<const uint4 *>(code)[p.base[n] + (uint32_t)u];
            const uint32_t op = pending ? (w.x & 0xffu) : (uint32_t)OP_STUCK;
            const uint32_t src = (w.x >> 8) & 0xffu;
            const bool dacc = ((w.x >> 16) & 0xffu) != 0u;
            const uint32_t arg = w.y & 0xffffu;
            const int64_t imm = (int64_t)(((uint64_t)w.w << 32) | (uint64_t)w.z);
            bool ret = false;             // retires: ip advances (or jumps), steps++
            int32_t tgt = -1;             // jump target when >= 0
            auto record = [&]() { // mk_trace_lane: one entry per retired instruction of input 0
                if (p.trace && idx == 0 && ntrace < p.trace_max) {
                    mk_trace_entry &e = p.trace[ntrace++];
                    e.round = round;
                    e.node = (uint16_t)n;
                    e.ip = (uint16_t)u;
                    e.acc = acc[n];
                    e.bak = bak[n];
                }
            };
            // ops without a source operand
            if (op == OP_NOP) ret = true;
            if (op == OP_SWP) { const int64_t t = acc[n]; acc[n] = bak[n]; bak[n] = t; ret = true; }
            if (op == OP_SAV) { bak[n] = acc[n]; ret = true; }
            if (op == OP_NEG) { acc[n] = (int64_t)(0ull - (uint64_t)acc[n]); ret = true; }
            if (op >= OP_JMP && op <= OP_JLZ) {
                const int64_t a = acc[n];
                const bool take = op == OP_JMP || (op == OP_JEZ && a == 0) || (op == OP_JNZ && a != 0) ||
                                  (op == OP_JGZ && a > 0) || (op == OP_JLZ && a < 0);
                ret = true;
                tgt = take ? (int32_t)arg : -1;
            }
            if (op == OP_IN && in_avail) { // <-m.inChan (master.go:235)
                in_avail = false;
                if (dacc) acc[n] = in_val;
                ret = true;
            }
            if (op == OP_POP) {
                int32_t *dp = &sdepth[arg * B + tid];
                const int32_t d = *dp;
                if (d > 0) { // waitPop blocks while empty (stack.go:133-155)
                    const uint32_t e = (uint32_t)d - 1;
                    int32_t *rp = &ring[(arg * W + (e & (W - 1))) * B + tid];
                    const int32_t v = *rp;
                    if (e >= W) *rp = p.spill[((uint64_t)arg * p.spill_rows + (e - W)) * p.lanes + gid];
                    *dp = (int32_t)e;
                    if (dacc) acc[n] = v;
                    ret = true;
                }
            }
            // ops with a source operand: getFromSrc (program.go:434-472)
            const bool srcop = op == OP_MOV || op == OP_ADD || op == OP_SUB || op == OP_JRO || op == OP_SEND ||
                               op == OP_OUT || op == OP_PUSH || op == OP_HANG || op == OP_RETRY;
            const bool pn = (pend >> n) & 1u;
            bool have = srcop, consumed = false;
            int64_t v = 0;
            if (srcop) {
                if (pn) v = pendv[n];
                else if (src == SRC_IMM) v = imm;
                else if (src == SRC_ACC) v = acc[n];
                else if (src >= SRC_R0) {
                    const uint32_t slot = (uint32_t)n * 4 + (src - SRC_R0);
                    if ((pfull >> slot) & 1ull) {
                        v = port[slot * B + tid];
                        pfull &= ~(1ull << slot);
                        consumed = true;
                    } else {
                        have = false; // receive blocks
                    }
                }
            }
            if (have) {
                if (op == OP_MOV) { if (dacc) acc[n] = v; ret = true; }
                if (op == OP_ADD) { acc[n] = (int64_t)((uint64_t)acc[n] + (uint64_t)v); ret = true; }
                if (op == OP_SUB) { acc[n] = (int64_t)((uint64_t)acc[n] - (uint64_t)v); ret = true; }
                if (op == OP_JRO) { // IntClamp(ptr+v, 0, len-1), int64 wrapping add (program.go:354,362)
                    int64_t t = (int64_t)((uint64_t)(int64_t)u + (uint64_t)v);
                    t = t > (int64_t)len - 1 ? (int64_t)len - 1 : t;
                    t = t < 0 ? 0 : t;
                    ret = true;
                    tgt = (int32_t)t;
                }
                if (op == OP_SEND) {
                    if (!((pfull >> arg) & 1ull)) { // p.rK <- int32(v) (program.go:163,498)
                        port[arg * B + tid] = (int32_t)v;
                        pfull |= 1ull << arg;
                        pend &= ~(1u << n);
                        ret = true;
                    } else if (!pn) {
                        pend |= 1u << n;
                        pendv[n] = (int32_t)v;
                        changed = true;
                    }
                }
                if (op == OP_OUT) {
                    if (out_cnt < 2) { // outChan cap 1 + one /compute read (master.go:219,246)
                        if (out_cnt == 0) out_val = (int32_t)v;
                        ++out_cnt;
                        pend &= ~(1u << n);
                        ret = true;
                        if (p.flags & MK_FLAG_STOP_ON_OUTPUT) { done = true; reason = MK_ST_OUTPUT_STOP; }
                    } else if (!pn) {
                        pend |= 1u << n;
                        pendv[n] = (int32_t)v;
                        changed = true;
                    }
                }
                if (op == OP_PUSH) {
                    int32_t *dp = &sdepth[arg * B + tid];
                    const uint32_t d = (uint32_t)*dp;
                    if (d >= p.stack_cap) {
                        done = true;
                        reason = MK_ST_STACK_OVERFLOW;
                    } else {
                        int32_t *rp = &ring[(arg * W + (d & (W - 1))) * B + tid];
                        if (d >= W) p.spill[((uint64_t)arg * p.spill_rows + (d - W)) * p.lanes + gid] = *rp;
                        *rp = (int32_t)v; // ValueMessage{int32(v)} (program.go:516)
                        *dp = (int32_t)(d + 1);
                        ret = true;
                    }
                }
                if (op == OP_HANG) { hung |= 1u << n; changed = true; }
                if (op == OP_RETRY && consumed) changed = true;
            }
            if (ret) {
                ip[n] = tgt >= 0 ? tgt : ((u + 1 == (int32_t)len) ? 0 : u + 1); // program.go:429
                ++steps;
                changed = true;
                record();
            }
        }
        if (active && !done) {
            if (!changed) { done = true; reason = MK_ST_QUIESCENT; }
            else if (steps >= p.budget) { done = true; reason = MK_ST_BUDGET; }
        }
        ++round;
        if (done && p.trace && idx == 0) *p.trace_n = ntrace;
        if (done) {
            const uint32_t st = reason | (out_cnt > 0 ? MK_ST_HAS_OUTPUT : 0u);
            p.out[idx] = out_cnt > 0 ? out_val : 0;
            p.status[idx] = (uint8_t)st;
            if (p.steps) p.steps[idx] = steps;
            s_steps += steps;
            s_out += out_cnt > 0;
            s_done += 1;
            s_q += reason == MK_ST_QUIESCENT;
            s_b += reason == MK_ST_BUDGET;
            s_ov += reason == MK_ST_STACK_OVERFLOW;
            s_os += reason == MK_ST_OUTPUT_STOP;
            idx += p.lanes;
            active = idx < p.n;
            if (active) init(idx);
        }
    }

    if (p.partials) {
        const unsigned long long c[7] = {s_steps, s_out, s_done, s_q, s_b, s_ov, s_os};
        write_partials(p.partials, gid, c);
    }
}

// ------------------------------------------------------------------------
// Tier 2: superblock executor for a compiled schedule (tis_sched.cpp).
//
// Each lane carries only its superblock id, its retired-instruction count
// and a small file of 64-bit registers in LDS ([reg][lane], conflict-free
// for every access); stack entries that outlive a superblock sit in HBM
// slots laid out [slot][lane] (coalesced).  A wave picks the superblock of
// its lowest active lane, runs the lanes that share it through the
// micro-op stream (scalar fetch + scalar dispatch, VALU only for the data),
// and repeats; lanes leave a superblock at BR/JRO/JUMP/END/GUARD/ROUND_END.
// ------------------------------------------------------------------------

// `i` must be wave-uniform.  readfirstlane pins the index and every fetched
// dword to SGPRs: the fetch is scalar loads and the opcode switch a scalar
// branch (without it the compiler loses uniformity through the dispatch loop
// and emits vector loads plus an exec-masked case chain).
// readfirstlane returns a signed int: keep every word unsigned so that no
// 32-bit half of an immediate is sign-extended into the other.
__device__ __forceinline__ uint32_t rfl(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }

__device__ __forceinline__ DOp fetch_dop(const DOp *__restrict__ code, uint32_t i)
{
    i = rfl(i);
    const uint4 *q = reinterpret_cast<const uint4 *>(code) + 2 * (size_t)i;
    const uint4 w0 = q[0], w1 = q[1];
    DOp o;
    o.op = rfl(w0.x);
    o.fl = rfl(w0.y);
    o.d = rfl(w0.z);
    o.a = rfl(w0.w);
    o.b = rfl(w1.x);
    o.inc = rfl(w1.y);
    o.imm = (int64_t)(((uint64_t)rfl(w1.w) << 32) | (uint64_t)rfl(w1.z));
    return o;
}


// ---- tier-2 superblock execution ------------------------------------------
// LDS register file layout: [reg][slot k][lane] int64, so register r of slot k
// for this lane sits at lane_base + r * (K * B * 8) + k * (B * 8).  DOp register
// operands are pre-scaled byte offsets r * K * B * 8 (assemble_device); with B
// a template constant the K slots of one register are one address computation
// plus immediate-offset ds_read/ds_write.

template <int K, int B>
struct Slots {
    char *lane_base;
    __device__ __forceinline__ int64_t *at(uint32_t off) const { return reinterpret_cast<int64_t *>(lane_base + off); }
};

__device__ __forceinline__ int64_t sx32(int64_t v, uint32_t t) { return t ? (int64_t)(int32_t)(uint32_t)(uint64_t)v : v; }

// Executes data micro-ops (MOV..LD) from `pc` and returns the first control
// op, leaving `pc` on it.  The loop carries nothing but `pc`.  FULL: every
// slot of the thread is in the group.  Otherwise slots outside the group
// compute too (reading stale registers is harmless) but their writes go to a
// scratch register / scratch HBM row -- selects instead of per-slot branches,
// so the loop never manipulates the exec mask.
template <int K, int B>
__device__ __forceinline__ void load_slots(const Slots<K, B> &S, uint32_t off, uint32_t t, int64_t (&v)[K])
{
    const int64_t *a = S.at(off);
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = a[k * B];
    if (t) {
#pragma unroll
        for (int k = 0; k < K; ++k) v[k] = (int64_t)(int32_t)(uint32_t)(uint64_t)v[k];
    }
}

template <int K, int B, bool FULL>
__device__ __forceinline__ DOp run_data(const DOp *__restrict__ code, uint32_t &pc, const SParams &p,
                                        const Slots<K, B> &S, uint64_t vlane0, const bool (&mine)[K])
{
    for (;;) {
        const DOp I = fetch_dop(code, pc);
        if (I.op > U_DATA_LAST) return I;
        if (I.op <= U_RSUBI) { // MOV LI ADD SUB ADDI RSUBI: int64 arithmetic on registers
            int64_t v[K];
            if (I.op == U_LI) {
#pragma unroll
                for (int k = 0; k < K; ++k) v[k] = I.imm;
            } else {
                load_slots<K, B>(S, I.a, I.fl & UF_TA, v);
                if (I.op == U_ADDI) {
#pragma unroll
                    for (int k = 0; k < K; ++k) v[k] = (int64_t)((uint64_t)v[k] + (uint64_t)I.imm);
                } else if (I.op == U_RSUBI) {
#pragma unroll
                    for (int k = 0; k < K; ++k) v[k] = (int64_t)((uint64_t)I.imm - (uint64_t)v[k]);
                } else if (I.op != U_MOV) {
                    int64_t w[K];
                    load_slots<K, B>(S, I.b, I.fl & UF_TB, w);
                    if (I.op == U_ADD) {
#pragma unroll
                        for (int k = 0; k < K; ++k) v[k] = (int64_t)((uint64_t)v[k] + (uint64_t)w[k]);
                    } else {
#pragma unroll
                        for (int k = 0; k < K; ++k) v[k] = (int64_t)((uint64_t)v[k] - (uint64_t)w[k]);
                    }
                }
            }
            if (FULL) {
                int64_t *d = S.at(I.d);
#pragma unroll
                for (int k = 0; k < K; ++k) d[k * B] = v[k];
            } else {
#pragma unroll
                for (int k = 0; k < K; ++k) S.at(mine[k] ? I.d : p.scratch_off)[k * B] = v[k];
            }
        } else if (I.op == U_LD) { // stack entry back from its HBM slot
            const int32_t *src = p.slots + (uint64_t)I.imm * p.vlanes + vlane0;
            int64_t v[K];
#pragma unroll
            for (int k = 0; k < K; ++k) v[k] = src[(uint64_t)k * p.lanes];
            if (FULL) {
                int64_t *d = S.at(I.d);
#pragma unroll
                for (int k = 0; k < K; ++k) d[k * B] = v[k];
            } else {
#pragma unroll
                for (int k = 0; k < K; ++k) S.at(mine[k] ? I.d : p.scratch_off)[k * B] = v[k];
            }
        } else if (I.op == U_LDX) { // dynamic stack: slot imm + R[b]
            int64_t x[K], v[K];
            load_slots<K, B>(S, I.b, 0, x);
#pragma unroll
            for (int k = 0; k < K; ++k) {
                // slots outside the group may hold any index: they read the scratch row
                const uint64_t row = (FULL || mine[k]) ? (uint64_t)I.imm + (uint64_t)x[k] : p.scratch_slot;
                v[k] = p.slots[row * p.vlanes + vlane0 + (uint64_t)k * p.lanes];
            }
            if (FULL) {
                int64_t *d = S.at(I.d);
#pragma unroll
                for (int k = 0; k < K; ++k) d[k * B] = v[k];
            } else {
#pragma unroll
                for (int k = 0; k < K; ++k) S.at(mine[k] ? I.d : p.scratch_off)[k * B] = v[k];
            }
        } else if (I.op == U_STX) {
            int64_t x[K], v[K];
            load_slots<K, B>(S, I.b, 0, x);
            load_slots<K, B>(S, I.a, I.fl & UF_TA, v);
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const uint64_t row = (FULL || mine[k]) ? (uint64_t)I.imm + (uint64_t)x[k] : p.scratch_slot;
                p.slots[row * p.vlanes + vlane0 + (uint64_t)k * p.lanes] = (int32_t)v[k];
            }
        } else { // ST / STI: stack entry to its HBM slot
            int64_t v[K];
            uint64_t slot;
            if (I.op == U_STI) {
                slot = I.d;
#pragma unroll
                for (int k = 0; k < K; ++k) v[k] = I.imm;
            } else {
                slot = (uint32_t)I.imm;
                load_slots<K, B>(S, I.a, I.fl & UF_TA, v);
            }
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const uint64_t row = (FULL || mine[k]) ? slot : p.scratch_slot;
                p.slots[row * p.vlanes + vlane0 + (uint64_t)k * p.lanes] = (int32_t)v[k];
            }
        }
        ++pc;
    }
}

// Applies control op E (JUMP/BR/JRO/END) to the slots in `mine` (selects).
template <int K, int B>
__device__ __forceinline__ void apply_exit(const DOp &E, const uint32_t *__restrict__ jtab, const Slots<K, B> &S,
                                           const bool (&mine)[K], uint32_t (&sb)[K], uint32_t (&steps)[K],
                                           bool (&done)[K], uint32_t (&st)[K], int32_t (&outv)[K])
{
    const uint32_t ta = E.fl & UF_TA;
    const int64_t *a = S.at(E.a);
    if (E.op == U_JUMP) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            steps[k] += mine[k] ? E.inc : 0u;
            sb[k] = mine[k] ? (uint32_t)E.imm : sb[k];
        }
    } else if (E.op == U_BR) {
        const uint32_t cond = (E.fl >> UF_COND_SHIFT) & 3u;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int64_t v = sx32(a[k * B], ta);
            const bool take = cond == 0 ? v == 0 : cond == 1 ? v != 0 : cond == 2 ? v > 0 : v < 0;
            steps[k] += mine[k] ? E.inc : 0u;
            const uint32_t nsb = take ? (uint32_t)(uint64_t)E.imm : (uint32_t)((uint64_t)E.imm >> 32);
            sb[k] = mine[k] ? nsb : sb[k];
        }
    } else if (E.op == U_END) {
        const bool outreg = (E.fl & UF_OUTREG) != 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            steps[k] += mine[k] ? E.inc : 0u;
            const int32_t o = outreg ? (int32_t)sx32(a[k * B], ta) : (int32_t)E.imm;
            outv[k] = mine[k] ? o : outv[k];
            st[k] = mine[k] ? E.d : st[k];
            done[k] = done[k] || mine[k];
        }
    } else if (E.op == U_JRO) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            // IntClamp(ptr+v, 0, len-1) with an int64 wrapping add (program.go:354,362)
            int64_t t = (int64_t)((uint64_t)E.d + (uint64_t)sx32(a[k * B], ta));
            t = t > (int64_t)E.b ? (int64_t)E.b : t;
            t = t < 0 ? 0 : t;
            steps[k] += mine[k] ? E.inc : 0u;
            if (mine[k]) sb[k] = jtab[(uint64_t)E.imm + (uint64_t)t];
        }
    } else { // corrupt stream: end the slots
#pragma unroll
        for (int k = 0; k < K; ++k) {
            st[k] = mine[k] ? 0u : st[k];
            done[k] = done[k] || mine[k];
        }
    }
}

// OVF (a PUSH onto a dynamic stack): the slots of the group whose depth
// register is at the limit end with the op's status.  Returns whether any
// slot of the wave is still in the group; `cut` = some slot left it.
template <int K, int B>
__device__ __forceinline__ bool apply_ovf(const DOp &E, const Slots<K, B> &S, bool (&mine)[K], uint32_t (&steps)[K],
                                          bool (&done)[K], uint32_t (&st)[K], int32_t (&outv)[K], bool &cut)
{
    const int64_t *a = S.at(E.a), *x = S.at(E.b);
    const uint64_t lim = (uint64_t)E.imm >> 32;
    bool left = false, stop_any = false;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const bool stop = mine[k] && (uint64_t)x[k * B] >= lim;
        const int32_t o = (E.fl & UF_OUTREG) ? (int32_t)sx32(a[k * B], E.fl & UF_TA) : (int32_t)(uint32_t)E.imm;
        steps[k] += stop ? E.inc : 0u;
        outv[k] = stop ? o : outv[k];
        st[k] = stop ? E.d : st[k];
        done[k] = done[k] || stop;
        mine[k] = mine[k] && !stop;
        left = left || mine[k];
        stop_any = stop_any || stop;
    }
    cut = __ballot(stop_any) != 0;
    return __ballot(left) != 0;
}

// BRX (an in-line side exit): the slots of the group whose condition holds
// leave for variant E.imm.  Returns whether any slot of the wave is still in
// the group; `cut` = some slot left it.
template <int K, int B>
__device__ __forceinline__ bool apply_brx(const DOp &E, const Slots<K, B> &S, bool (&mine)[K], uint32_t (&sb)[K],
                                          uint32_t (&steps)[K], bool &cut)
{
    const int64_t *a = S.at(E.a);
    const uint32_t cond = (E.fl >> UF_COND_SHIFT) & 3u;
    bool left = false, go_any = false;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int64_t v = sx32(a[k * B], E.fl & UF_TA);
        const bool take = cond == 0 ? v == 0 : cond == 1 ? v != 0 : cond == 2 ? v > 0 : v < 0;
        const bool go = mine[k] && take;
        steps[k] += go ? E.inc : 0u;
        sb[k] = go ? (uint32_t)E.imm : sb[k];
        mine[k] = mine[k] && !go;
        left = left || mine[k];
        go_any = go_any || go;
    }
    cut = __ballot(go_any) != 0;
    return __ballot(left) != 0;
}

// Budget-checked variant (taken only by groups that could reach the budget
// inside a superblock): ROUND_END and OVF may stop single slots, BRX move
// them to another variant.
template <int K, int B>
__device__ void run_checked(const DOp *__restrict__ code, const uint32_t *__restrict__ jtab, uint32_t pc,
                            const SParams &p, const Slots<K, B> &S, uint64_t vlane0, bool (&mine)[K],
                            uint32_t (&sb)[K], uint32_t (&steps)[K], bool (&done)[K], uint32_t (&st)[K],
                            int32_t (&outv)[K])
{
    for (;;) {
        const DOp E = run_data<K, B, false>(code, pc, p, S, vlane0, mine);
        if (E.op == U_ROUND_END) {
            const int64_t *a = S.at(E.a);
            bool left = false;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const bool stop = mine[k] && (uint64_t)steps[k] + E.inc >= p.budget;
                const int32_t o = (E.fl & UF_OUTREG) ? (int32_t)sx32(a[k * B], E.fl & UF_TA) : (int32_t)E.imm;
                steps[k] += stop ? E.inc : 0u;
                outv[k] = stop ? o : outv[k];
                st[k] = stop ? E.d : st[k];
                done[k] = done[k] || stop;
                mine[k] = mine[k] && !stop;
                left = left || mine[k];
            }
            if (!__ballot(left)) return;
            ++pc;
            continue;
        }
        if (E.op == U_OVF) {
            bool cut;
            if (!apply_ovf<K, B>(E, S, mine, steps, done, st, outv, cut)) return;
            ++pc;
            continue;
        }
        if (E.op == U_BRX) {
            bool cut;
            if (!apply_brx<K, B>(E, S, mine, sb, steps, cut)) return;
            ++pc;
            continue;
        }
        apply_exit<K, B>(E, jtab, S, mine, sb, steps, done, st, outv);
        return;
    }
}

// One waterfall step of a wave: the superblock u of the first active slot of
// the wave is run for every slot sitting on it ("the group").  A scalar fetch
// and dispatch of each micro-op serves all K x 64 slots of the group.  fin[k]
// is set for slots that ended in this step; st/outv are written for them only.
// Returns false (wave-uniform) once no slot of the wave is active.
template <int K, int B>
__device__ __forceinline__ bool sched_step(const DOp *__restrict__ code, const uint32_t *__restrict__ entry,
                                           const uint32_t *__restrict__ jtab, const SParams &p,
                                           const Slots<K, B> &S, uint64_t gid, const bool (&act)[K],
                                           uint32_t (&sb)[K], uint32_t (&steps)[K], bool (&fin)[K],
                                           uint32_t (&st)[K], int32_t (&outv)[K])
{
    bool any = false;
    uint32_t fsb = 0;
#pragma unroll
    for (int k = K - 1; k >= 0; --k) {
        any = any || act[k];
        if (act[k]) fsb = sb[k];
        fin[k] = false;
    }
    const unsigned long long anyb = __ballot(any);
    if (!anyb) return false;
    const uint32_t u = rfl((uint32_t)__builtin_amdgcn_readlane((int)fsb, __builtin_ctzll(anyb)));
    bool mine[K], mine_any = false, mine_all = true;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        mine[k] = act[k] && sb[k] == u;
        mine_any = mine_any || mine[k];
        mine_all = mine_all && mine[k];
    }
    bool full = __ballot(mine_any && !mine_all) == 0;
    if (!mine_any) return true;
    uint32_t pc = rfl(entry[u]);
    if (u & 1u) {
        run_checked<K, B>(code, jtab, pc, p, S, gid, mine, sb, steps, fin, st, outv);
        return true;
    }
    for (;;) {
        const DOp E = full ? run_data<K, B, true>(code, pc, p, S, gid, mine)
                           : run_data<K, B, false>(code, pc, p, S, gid, mine);
        if (E.op == U_GUARD) {
            // any slot that could reach the budget inside: the whole group
            // takes the checked variant (exact for every slot)
            bool need = false;
#pragma unroll
            for (int k = 0; k < K; ++k) need = need || (mine[k] && (uint64_t)steps[k] + E.inc >= p.budget);
            if (__ballot(need)) {
#pragma unroll
                for (int k = 0; k < K; ++k) sb[k] = mine[k] ? (uint32_t)E.imm : sb[k];
                return true;
            }
            ++pc;
            continue;
        }
        if (E.op == U_OVF) {
            bool cut;
            if (!apply_ovf<K, B>(E, S, mine, steps, fin, st, outv, cut)) return true;
            full = full && !cut;
            ++pc;
            continue;
        }
        if (E.op == U_BRX) {
            bool cut;
            if (!apply_brx<K, B>(E, S, mine, sb, steps, cut)) return true;
            full = full && !cut;
            ++pc;
            continue;
        }
        apply_exit<K, B>(E, jtab, S, mine, sb, steps, fin, st, outv);
        return true;
    }
}


// Refill scheduling: slot k of thread gid runs inputs gid + k*lanes, then
// + vlanes, ...; a slot that finishes writes its result and immediately takes
// its next input (prefetched one input ahead).
template <int K, int B>
__global__ void __launch_bounds__(B) tis_sched_exec(const DOp *__restrict__ code, const uint32_t *__restrict__ entry,
                                                    const uint32_t *__restrict__ jtab, SParams p)
{
    extern __shared__ int64_t R[]; // [nregs][K][B]
    const uint32_t tid = threadIdx.x;
    const uint64_t gid = (uint64_t)blockIdx.x * B + tid;
    const Slots<K, B> S{reinterpret_cast<char *>(R) + tid * 8};
    const uint64_t stride = p.vlanes; // inputs per round of all slots

    unsigned long long cnt[7] = {0, 0, 0, 0, 0, 0, 0}; // steps, out, done, quiescent, budget, overflow, out-stop
    uint64_t idx[K];
    bool act[K], fin[K];
    uint32_t sb[K], steps[K], st[K];
    int32_t nxt[K], outv[K];
    int64_t *in_reg = S.at(p.in_off);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        idx[k] = gid + (uint64_t)k * p.lanes;
        act[k] = idx[k] < p.n;
        sb[k] = 0;
        steps[k] = 0;
        st[k] = 0;
        outv[k] = 0;
        nxt[k] = 0;
        if (act[k]) {
            in_reg[k * B] = sched_input(p, idx[k]);
            if (idx[k] + stride < p.n) nxt[k] = sched_input(p, idx[k] + stride);
        }
    }
    while (sched_step<K, B>(code, entry, jtab, p, S, gid, act, sb, steps, fin, st, outv)) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (!fin[k]) continue;
            p.out[idx[k]] = (st[k] & MK_ST_HAS_OUTPUT) ? outv[k] : 0;
            p.status[idx[k]] = (uint8_t)st[k];
            if (p.steps) p.steps[idx[k]] = steps[k];
            count_lane(cnt, steps[k], st[k]);
            idx[k] += stride;
            act[k] = idx[k] < p.n;
            sb[k] = 0;
            steps[k] = 0;
            if (act[k]) {
                in_reg[k * B] = nxt[k];
                if (idx[k] + stride < p.n) nxt[k] = sched_input(p, idx[k] + stride);
            }
        }
    }
    if (p.partials) write_partials(p.partials, gid, cnt);
}

// K contiguous inputs at `base` (ragged tail: only those < n).
template <int K>
__device__ __forceinline__ void tile_inputs(const SParams &p, uint64_t base, int32_t (&v)[K])
{
    if (p.io_vec && base + K <= p.n) {
        const int32_t *src = (const int32_t *)p.in_data + base;
        if constexpr (K == 4) {
            const int4 q = *reinterpret_cast<const int4 *>(src);
            v[0] = q.x, v[1] = q.y, v[2] = q.z, v[3] = q.w;
        } else if constexpr (K == 2) {
            const int2 q = *reinterpret_cast<const int2 *>(src);
            v[0] = q.x, v[1] = q.y;
        } else {
            v[0] = src[0];
        }
        return;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = base + k < p.n ? sched_input(p, base + k) : 0;
}

// Tile scheduling: a block takes tiles of K*B contiguous inputs (grid-stride),
// thread tid owns inputs base = tile*K*B + tid*K .. base+K-1, the next tile's
// inputs are loaded while this one runs, and results leave in vector stores
// once every lane of the tile has finished.
template <int K, int B>
__global__ void __launch_bounds__(B) tis_sched_tile(const DOp *__restrict__ code, const uint32_t *__restrict__ entry,
                                                    const uint32_t *__restrict__ jtab, SParams p)
{
    extern __shared__ int64_t R[]; // [nregs][K][B]
    const uint32_t tid = threadIdx.x;
    const uint64_t gid = (uint64_t)blockIdx.x * B + tid;
    const Slots<K, B> S{reinterpret_cast<char *>(R) + tid * 8};
    const uint64_t tile = (uint64_t)K * B, ntiles = (p.n + tile - 1) / tile;

    unsigned long long cnt[7] = {0, 0, 0, 0, 0, 0, 0};
    int64_t *in_reg = S.at(p.in_off);
    int32_t nxt[K];
    uint64_t t = blockIdx.x;
    if (t < ntiles) tile_inputs<K>(p, t * tile + (uint64_t)tid * K, nxt);
    for (; t < ntiles; t += gridDim.x) {
        const uint64_t base = t * tile + (uint64_t)tid * K;
        bool act[K], fin[K];
        uint32_t sb[K], steps[K], st[K];
        int32_t outv[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            act[k] = base + k < p.n;
            sb[k] = 0;
            steps[k] = 0;
            st[k] = 0;
            outv[k] = 0;
            in_reg[k * B] = nxt[k];
        }
        if (t + gridDim.x < ntiles) tile_inputs<K>(p, base + (uint64_t)gridDim.x * tile, nxt);
        while (sched_step<K, B>(code, entry, jtab, p, S, gid, act, sb, steps, fin, st, outv)) {
#pragma unroll
            for (int k = 0; k < K; ++k) act[k] = act[k] && !fin[k];
        }
#pragma unroll
        for (int k = 0; k < K; ++k) outv[k] = (st[k] & MK_ST_HAS_OUTPUT) ? outv[k] : 0;
        if (p.io_vec && base + K <= p.n) {
            if constexpr (K == 4) {
                *reinterpret_cast<int4 *>(p.out + base) = make_int4(outv[0], outv[1], outv[2], outv[3]);
                *reinterpret_cast<uint32_t *>(p.status + base) =
                    (st[0] & 0xffu) | (st[1] & 0xffu) << 8 | (st[2] & 0xffu) << 16 | st[3] << 24;
                if (p.steps)
                    *reinterpret_cast<uint4 *>(p.steps + base) = make_uint4(steps[0], steps[1], steps[2], steps[3]);
            } else if constexpr (K == 2) {
                *reinterpret_cast<int2 *>(p.out + base) = make_int2(outv[0], outv[1]);
                *reinterpret_cast<uint16_t *>(p.status + base) = (uint16_t)((st[0] & 0xffu) | (st[1] & 0xffu) << 8);
                if (p.steps) *reinterpret_cast<uint2 *>(p.steps + base) = make_uint2(steps[0], steps[1]);
            } else {
                p.out[base] = outv[0];
                p.status[base] = (uint8_t)st[0];
                if (p.steps) p.steps[base] = steps[0];
            }
        } else {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                if (base + k >= p.n) continue;
                p.out[base + k] = outv[k];
                p.status[base + k] = (uint8_t)st[k];
                if (p.steps) p.steps[base + k] = steps[k];
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (base + k < p.n) count_lane(cnt, steps[k], st[k]);
    }
    if (p.partials) write_partials(p.partials, gid, cnt);
}

// ------------------------------------------------------------------------
// Stateful sessions.
//
// The reference's nodes keep running between /compute calls (program.go:
// 80-92): ACC, BAK, ptr, ports, stacks and the master's inChan / outChan
// (capacity 1 each, master.go:58-59) persist.  A session set is n network
// instances whose state lives in HBM between calls (struct of arrays,
// [field][session], coalesced); tis_session runs one /compute call on every
// session, one thread each (oracle: tis_oracle.c session_call):
//   loop: deposit the input once inChan is empty (m.inChan <- v, :216);
//         take outChan's value once the input is deposited (:219) -> result;
//         end the slice at the budget; run one round; a stack overflow or a
//         round without change ends the call.
// A call whose slice reaches the budget stays open (MK_ST_BUDGET) and a
// resume launch continues it; a round without change closes it without a
// result and the instance lives on; a stack overflow ends the session.
// Ports are staged in LDS for the call; stack entries stay in HBM.
// ------------------------------------------------------------------------
struct SessImport {
    uint64_t n;
    int nprog, nstack;
    uint32_t *nsb;
    uint32_t *sflags;   // SessParams::sflags (written here)
    uint32_t epoch;     // this launch (the native kernel stores it into sflags[0] at a hand-off)
    const uint32_t *hand_sb, *hand_steps;
    const int64_t *regs;  // [register][n]
    const int32_t *slots; // [slot][n]
    const SessMapHdr *hdr;
    const SessSrcDev *rec;
    const int64_t *dyn_base;
};

struct SessParams {
    uint32_t base[MK_MAX_PROGRAM_NODES];
    uint32_t len[MK_MAX_PROGRAM_NODES];
    int nprog;
    int nstack;
    uint64_t n;         // sessions
    uint32_t budget;    // retired instructions per call
    uint32_t stack_cap;
    uint32_t ncalls;    // sequential /compute calls per session in this launch
    const int64_t *in;  // [ncalls][n] the calls' inputs (strconv.Atoi values)
    int32_t *out;       // [ncalls][n]
    uint8_t *status;    // [ncalls][n]
    uint32_t *steps;    // [ncalls][n] or null
    int64_t *acc, *bak; // [nprog][n]
    int32_t *ip, *pendv;  // [nprog][n]
    int32_t *port;      // [nprog*4][n]
    uint64_t *pfull;    // [n]
    uint32_t *bits;     // [n]: pend (bits 0-15) | hung (bits 16-31)
    uint32_t *io;       // [n]: in_full | out_full << 1 | dead << 4
    int32_t *in_val, *out_val; // [n]
    int32_t *sdepth;    // [nstack][n]
    int32_t *stk;       // [nstack][stack_cap][n]
    // remote peers (MK_NODE_REMOTE_*, row f4): per program node, the state of
    // its request to a peer (0 none, 1 asked, 2 answered by the host) and the
    // value (sent, pushed, or popped); a call parked on them resumes
    uint32_t *xst;      // [nprog][n]
    int32_t *xval;      // [nprog][n]
    int32_t *pin;       // [n] input of the current call not yet deposited
    uint32_t *csteps;   // [n] steps retired by the current call so far
    uint32_t mixed;     // network has remote peers: a round without change parks the call
    uint32_t resume;    // continue each session's parked call (in ignored)
    // native sessions (tis_jit.h mk_sess_exec): the interpreter runs only the
    // sessions marked MK_SS_T1 here (null: all).  One handed off in this
    // launch (io bit 8, set by sess_import_one) starts at its call
    // hand_call[i], resumed, its step count that of the native slice, at
    // round position io bits 9-13 with io bit 14 "something changed".
    const uint32_t *nsb;       // [n]
    const uint32_t *hand_call; // [n]
    // [0] launch epoch of the last hand-off, [1] sessions the interpreter
    // holds (sess_import_one counts them): with none and no resume this
    // kernel has nothing to do
    const uint32_t *sflags;
    // the hand-off import, done by this kernel before it runs (one launch
    // fewer per call than round 3's separate import kernel)
    uint32_t fuse_import;
    SessImport imp;
};

struct SessImportOut {
    const SessParams &p;
    uint64_t i, n;
    uint32_t io = 0;
    __device__ void acc(int k, int64_t v) { p.acc[(uint64_t)k * n + i] = v; }
    __device__ void bak(int k, int64_t v) { p.bak[(uint64_t)k * n + i] = v; }
    __device__ void ip(int k, int32_t v) { p.ip[(uint64_t)k * n + i] = v; }
    __device__ void pendv(int k, int32_t v) { p.pendv[(uint64_t)k * n + i] = v; }
    __device__ void port(int q, int32_t v) { p.port[(uint64_t)q * n + i] = v; }
    __device__ void pfull(uint64_t x) { p.pfull[i] = x; }
    __device__ void bits(uint32_t pend, uint32_t hung) { p.bits[i] = (pend & 0xffffu) | (hung << 16); }
    __device__ void chans(bool in_full, bool out_full, int32_t iv, int32_t ov)
    {
        io |= (in_full ? 1u : 0u) | (out_full ? 2u : 0u);
        p.in_val[i] = iv;
        p.out_val[i] = ov;
    }
    __device__ void depth(int s, uint32_t d) { p.sdepth[(uint64_t)s * n + i] = (int32_t)d; }
    __device__ void entry(int s, uint32_t d, int32_t v) { p.stk[((uint64_t)s * p.stack_cap + d) * n + i] = v; }
    __device__ void call(bool dep, int32_t pin, int pos, bool changed)
    {
        io |= 8u | 0x100u | (dep ? 0u : 4u) | ((uint32_t)pos << 9) | (changed ? 0x4000u : 0u);
        p.pin[i] = pin;
    }
};

// One session's hand-off import (the native kernel's state at a HANDOFF into
// the interpreter's arrays, sess_convert.h), done by the
// interpreter kernel itself first (SessParams::fuse_import).
__device__ __forceinline__ void sess_import_one(const SessImport &q, const SessParams &p, uint64_t gid)
{
    if (gid >= q.n || q.nsb[gid] != kSessHand) return;
    const SessMapHdr h = q.hdr[q.hand_sb[gid]];
    const uint64_t n = q.n;
    auto reg = [&](uint32_t r) { return q.regs[(uint64_t)r * n + gid]; };
    auto slot = [&](uint32_t s) { return q.slots[(uint64_t)s * n + gid]; };
    SessImportOut o{p, gid, n};
    sess_convert(q.nprog, q.nstack, h, q.rec + h.off, q.dyn_base, reg, slot, o);
    p.io[gid] = o.io;
    p.csteps[gid] = q.hand_steps[gid];
    q.nsb[gid] = kSessT1;
    atomicAdd(&q.sflags[1], 1u);
}

// One session instance (gid) of the interpreter kernel below; `handed`: the
// native tier handed calls off in this launch, to be imported first.
template <int NMAX>
__device__ __forceinline__ void tis_session_one(const Insn *__restrict__ code, const SessParams &p, const uint64_t gid,
                                                int32_t *const lds, const bool handed)
{
    const int B = kBlock;
    const int tid = threadIdx.x;
    const uint64_t n = p.n;
    int32_t *const port = lds;                     // [nprog*4][B]
    int32_t *const sdepth = lds + p.nprog * 4 * B; // [nstack][B]
    if (handed) sess_import_one(p.imp, p, gid);
    const bool live = gid < n && (!p.nsb || p.nsb[gid] == kSessT1);

    int64_t acc[NMAX], bak[NMAX];
    int32_t ip[NMAX], pendv[NMAX], xval[NMAX];
    uint32_t xst[NMAX];
    uint64_t pfull = 0;
    uint32_t pend = 0, hung = 0, io = 0;
    int32_t in_val = 0, out_val = 0;
#pragma unroll
    for (int k = 0; k < NMAX; ++k) {
        const bool on = live && k < p.nprog;
        acc[k] = on ? p.acc[(uint64_t)k * n + gid] : 0;
        bak[k] = on ? p.bak[(uint64_t)k * n + gid] : 0;
        ip[k] = on ? p.ip[(uint64_t)k * n + gid] : 0;
        pendv[k] = on ? p.pendv[(uint64_t)k * n + gid] : 0;
        xst[k] = on && p.mixed ? p.xst[(uint64_t)k * n + gid] : 0u;
        xval[k] = on && p.mixed ? p.xval[(uint64_t)k * n + gid] : 0;
    }
    if (live) {
        for (int q = 0; q < p.nprog * 4; ++q) port[q * B + tid] = p.port[(uint64_t)q * n + gid];
        for (int q = 0; q < p.nstack; ++q) sdepth[q * B + tid] = p.sdepth[(uint64_t)q * n + gid];
        pfull = p.pfull[gid];
        const uint32_t bits = p.bits[gid];
        pend = bits & 0xffffu;
        hung = bits >> 16;
        io = p.io[gid];
        in_val = p.in_val[gid];
        out_val = p.out_val[gid];
    }
    bool in_full = io & 1u, out_full = (io >> 1) & 1u;
    uint32_t dead = (io >> 4) & 15u;
    const bool fresh = live && ((io >> 8) & 1u); // handed off by the native tier in this launch
    const uint32_t c0 = fresh ? p.hand_call[gid] : 0u;
    // ncalls sequential /compute calls, the state carried in registers/LDS
    // from one to the next (a burst of requests on one instance, one launch)
    for (uint32_t call = 0; call < p.ncalls; ++call) {
    const uint64_t ci = (uint64_t)call * n + gid;
    // io bit 3: a call is open (it parked on peers or ran out of its slice's
    // budget); bit 2: its input is not deposited yet (held in pin).  A resume
    // continues it with its input and step count; a new call while one is
    // open does nothing and reports MK_ST_CALL_OPEN (tis_oracle.c session_step)
    const bool open = live && ((io >> 3) & 1u);
    // a call the native tier handed off continues here (its earlier calls
    // of the burst were answered by the native kernel)
    const bool handed = fresh && call == c0, skip = fresh && call < c0;
    const bool resumed = (p.resume || handed) && open;
    const bool ran = live && !skip && dead == 0 && (p.resume || handed ? resumed : !open);
    const int32_t x = !live ? 0 : resumed ? p.pin[gid] : (int32_t)p.in[ci]; // int32(v) at GetInput (master.go:237)
    bool active = ran, got = false;
    bool deposited = resumed && !((io >> 2) & 1u);
    int32_t result = 0;
    uint32_t steps = resumed ? p.csteps[gid] : 0u;
    const uint32_t slice0 = handed ? 0u : steps; // a handed-off call is still in its first slice
    bool parked = false; // the call stays open
    uint32_t reason = 0;
    // where the hand-off stood inside a round: finish that round first
    int first_pos = handed ? (int)((io >> 9) & 31u) : 0;
    bool first_changed = handed && ((io >> 14) & 1u);

    for (;;) {
        if (active && first_pos == 0) {
            if (!deposited && !in_full) {
                in_full = true;
                in_val = x;
                deposited = true;
            }
            if (deposited && out_full) {
                out_full = false;
                result = out_val;
                got = true;
                active = false;
            } else if (steps - slice0 >= p.budget) { // this slice is spent; the call stays open
                reason = MK_ST_BUDGET;
                parked = true;
                active = false;
            }
        }
        if (!__ballot(active)) break;
        bool changed = first_changed, over = false;
        const int pos0 = first_pos;
        first_pos = 0;
        first_changed = false;
#pragma unroll
        for (int k = 0; k < NMAX; ++k) {
            if (k >= p.nprog) continue; // wave-uniform
            const uint32_t len = p.len[k];
            bool pending = active && !over && !((hung >> k) & 1u) && k >= pos0;
            unsigned long long todo = __ballot(pending);
            while (todo) {
                const int lead = __builtin_ctzll(todo);
                const int u = __builtin_amdgcn_readlane(ip[k], lead);
                const bool mine = pending && ip[k] == u;
                todo &= ~__ballot(mine);
                const Insn I = fetch(code, p.base[k] + (uint32_t)u);
                if (!mine) continue;
                pending = false;
                auto retire = [&]() {
                    ip[k] = (ip[k] + 1 == (int32_t)len) ? 0 : ip[k] + 1; // program.go:429
                    ++steps;
                    changed = true;
                };
                auto jump = [&](int32_t t) {
                    ip[k] = t;
                    ++steps;
                    changed = true;
                };
                switch (I.op) {
                case OP_NOP: retire(); break;
                case OP_SWP: { const int64_t t = acc[k]; acc[k] = bak[k]; bak[k] = t; retire(); break; }
                case OP_SAV: bak[k] = acc[k]; retire(); break;
                case OP_NEG: acc[k] = (int64_t)(0ull - (uint64_t)acc[k]); retire(); break;
                case OP_JMP: jump(I.arg); break;
                case OP_JEZ: if (acc[k] == 0) jump(I.arg); else retire(); break;
                case OP_JNZ: if (acc[k] != 0) jump(I.arg); else retire(); break;
                case OP_JGZ: if (acc[k] > 0) jump(I.arg); else retire(); break;
                case OP_JLZ: if (acc[k] < 0) jump(I.arg); else retire(); break;
                case OP_STUCK: break;
                case OP_XPOP: // popValue on a remote stack (program.go:524-536): the host makes the RPC
                    if (xst[k] == 2u) {
                        if (I.dst) acc[k] = xval[k];
                        xst[k] = 0u;
                        retire();
                    } else if (xst[k] == 0u) {
                        xst[k] = 1u;
                        changed = true;
                    }
                    break;
                case OP_IN:
                    if (in_full) { // <-m.inChan (master.go:235)
                        in_full = false;
                        if (I.dst) acc[k] = in_val;
                        retire();
                    }
                    break;
                case OP_POP: {
                    int32_t *dp = &sdepth[I.arg * B + tid];
                    const int32_t d = *dp;
                    if (d > 0) { // waitPop blocks while empty (stack.go:133-155)
                        const int32_t v = p.stk[((uint64_t)I.arg * p.stack_cap + (uint32_t)(d - 1)) * n + gid];
                        *dp = d - 1;
                        if (I.dst) acc[k] = v;
                        retire();
                    }
                    break;
                }
                default: {
                    // Ops with a source operand: getFromSrc (program.go:434-472).
                    const bool pn = (pend >> k) & 1u;
                    int64_t v = 0;
                    bool consumed = false;
                    if (pn) {
                        v = pendv[k];
                    } else if (I.src == SRC_IMM) {
                        v = I.imm;
                    } else if (I.src == SRC_ACC) {
                        v = acc[k];
                    } else if (I.src >= SRC_R0) {
                        const uint32_t slot = (uint32_t)k * 4 + (I.src - SRC_R0);
                        if (!((pfull >> slot) & 1ull)) break; // receive blocks
                        v = port[slot * B + tid];
                        pfull &= ~(1ull << slot);
                        consumed = true;
                    }
                    switch (I.op) {
                    case OP_MOV: if (I.dst) acc[k] = v; retire(); break;
                    case OP_ADD: acc[k] = (int64_t)((uint64_t)acc[k] + (uint64_t)v); retire(); break;
                    case OP_SUB: acc[k] = (int64_t)((uint64_t)acc[k] - (uint64_t)v); retire(); break;
                    case OP_JRO: {
                        int64_t t = (int64_t)((uint64_t)(int64_t)ip[k] + (uint64_t)v);
                        t = t > (int64_t)len - 1 ? (int64_t)len - 1 : t;
                        t = t < 0 ? 0 : t;
                        jump((int32_t)t);
                        break;
                    }
                    case OP_SEND: {
                        const uint32_t slot = I.arg;
                        if (!((pfull >> slot) & 1ull)) {
                            port[slot * B + tid] = (int32_t)v;
                            pfull |= 1ull << slot;
                            pend &= ~(1u << k);
                            retire();
                        } else if (!pn) {
                            pend |= 1u << k;
                            pendv[k] = (int32_t)v;
                            changed = true;
                        }
                        break;
                    }
                    case OP_OUT: // outChan <- v blocks while full (master.go:246)
                        if (!out_full) {
                            out_full = true;
                            out_val = (int32_t)v;
                            pend &= ~(1u << k);
                            retire();
                        } else if (!pn) {
                            pend |= 1u << k;
                            pendv[k] = (int32_t)v;
                            changed = true;
                        }
                        break;
                    case OP_PUSH: {
                        int32_t *dp = &sdepth[I.arg * B + tid];
                        const uint32_t d = (uint32_t)*dp;
                        if (d >= p.stack_cap) { over = true; break; }
                        p.stk[((uint64_t)I.arg * p.stack_cap + d) * n + gid] = (int32_t)v; // int32(v), program.go:516
                        *dp = (int32_t)(d + 1);
                        retire();
                        break;
                    }
                    case OP_HANG: hung |= 1u << k; changed = true; break;
                    case OP_RETRY: if (consumed) changed = true; break;
                    case OP_XSEND: case OP_XPUSH: // sendValue / pushValue to a peer (program.go:475-521)
                        if (xst[k] == 2u) { // the host's RPC returned
                            xst[k] = 0u;
                            pend &= ~(1u << k);
                            retire();
                        } else if (xst[k] == 0u) { // source fetched once, held as the pending value
                            pend |= 1u << k;
                            pendv[k] = (int32_t)v;
                            xval[k] = (int32_t)v; // int32(v) on the wire (program.go:498,516)
                            xst[k] = 1u;
                            changed = true;
                        }
                        break;
                    default: break;
                    }
                    break;
                }
                }
            }
        }
        if (active) {
            if (over) { // stack_cap (ours; the reference's stacks are unbounded) ends the session
                dead = reason = MK_ST_STACK_OVERFLOW;
                active = false;
            } else if (!changed) {
                // waits on peers or on the host's inbound RPCs: stays open;
                // otherwise nothing can change without another input -- the
                // call closes and the instance lives on
                if (p.mixed) parked = true, reason = MK_ST_REMOTE_WAIT;
                else reason = MK_ST_QUIESCENT;
                active = false;
            }
        }
    }
    if (live && !skip) {
        p.out[ci] = got ? result : 0;
        p.status[ci] = (uint8_t)(got ? MK_ST_HAS_OUTPUT : ran ? reason : dead ? dead : open && !p.resume ? MK_ST_CALL_OPEN : 0u);
        if (p.steps) p.steps[ci] = ran ? steps : 0u;
        if (ran) { // the call stays open while parked: input not yet deposited (bit 2), call open (bit 3)
            io = (io & ~0xCu) | (parked && !deposited ? 4u : 0u) | (parked ? 8u : 0u);
            if (parked) {
                p.pin[gid] = x;
                p.csteps[gid] = steps;
            }
        }
    } else if (gid < n && p.nsb && p.resume) {
        // a resume launch runs only this kernel: sessions the native tier
        // holds never have a call open (a budget slice hands the call to this
        // kernel), so there is nothing to resume -- or the session ended
        // (tis_oracle.c session_step)
        p.out[ci] = 0;
        p.status[ci] = p.nsb[gid] == kSessDead ? (uint8_t)MK_ST_STACK_OVERFLOW : (uint8_t)0;
        if (p.steps) p.steps[ci] = 0u;
    }
    } // calls

    if (!live) return;
#pragma unroll
    for (int k = 0; k < NMAX; ++k) {
        if (k >= p.nprog) continue;
        p.acc[(uint64_t)k * n + gid] = acc[k];
        p.bak[(uint64_t)k * n + gid] = bak[k];
        p.ip[(uint64_t)k * n + gid] = ip[k];
        p.pendv[(uint64_t)k * n + gid] = pendv[k];
    }
    if (p.mixed) {
#pragma unroll
        for (int k = 0; k < NMAX; ++k) {
            if (k >= p.nprog) continue;
            p.xst[(uint64_t)k * n + gid] = xst[k];
            p.xval[(uint64_t)k * n + gid] = xval[k];
        }
    }
    for (int q = 0; q < p.nprog * 4; ++q) p.port[(uint64_t)q * n + gid] = port[q * B + tid];
    for (int q = 0; q < p.nstack; ++q) p.sdepth[(uint64_t)q * n + gid] = sdepth[q * B + tid];
    p.pfull[gid] = pfull;
    p.bits[gid] = (pend & 0xffffu) | (hung << 16);
    p.io[gid] = (in_full ? 1u : 0u) | (out_full ? 2u : 0u) | (io & 0xCu) | (dead << 4);
    p.in_val[gid] = in_val;
    p.out_val[gid] = out_val;
}

// The interpreter over the session set, grid-stride: the grid is capped
// (kSessGridCap blocks), so a launch in which every session is the native
// tier's -- the common case, each thread leaving at the flag test -- costs
// a small grid instead of one block per 256 sessions (round 4: the per-call
// launch pair's second half).
template <int NMAX>
__global__ void __launch_bounds__(kBlock) tis_session(const Insn *__restrict__ code, SessParams p)
{
    extern __shared__ int32_t lds[];
    bool handed = false;
    if (p.fuse_import) {
        handed = p.imp.sflags[0] == p.imp.epoch; // something was handed off in this launch
        if (!handed && !p.resume && p.sflags[1] == 0u) return; // every session is the native tier's
    } else if (p.nsb && !p.resume && p.sflags[1] == 0u) {
        return; // every session is the native tier's
    }
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    const uint64_t end = (p.n + kBlock - 1) / kBlock * kBlock; // whole blocks: every thread takes the same trips
    for (uint64_t gid = (uint64_t)blockIdx.x * kBlock + threadIdx.x; gid < end; gid += stride)
        tis_session_one<NMAX>(code, p, gid, lds, handed);
}

// mk_session_cancel: abandon every open call (io bits 2-3); the state the
// call left behind -- its input if deposited, the nodes' progress -- stays.
__global__ void __launch_bounds__(kBlock) tis_session_cancel(uint32_t *io, uint64_t n)
{
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) io[i] &= ~0xCu;
}

// Native sessions handed off in this launch (MK_SS_HAND: a call's budget
// slice ends inside a superblock) become interpreter sessions: the state
// map of that superblock's entry (tis_sched.h SessMapHdr, from the schedule
// compiler) with the lane's registers and stack slots, in the interpreter's
// arrays (sess_convert.h), the call open and continuing its slice.



// ---- input order for the machine shape (tier 3) -----------------------------
// A wave of the machine-shape kernel runs 64 lanes together and each
// data-dependent loop until the wave's longest trip: lanes with similar
// inputs, whose trips are similar, waste less.  Before such a launch the
// input indices are grouped by value -- a counting sort into kOrderBuckets
// buckets over [min, max] of the batch -- and lane j answers input order[j].
// Every input is still evaluated exactly once and answered at its own index:
// only which lanes share a wave changes.
constexpr uint32_t kOrderBuckets = 4096;
constexpr uint64_t kOrderMin = 65536; // smaller batches launch unordered

__device__ __forceinline__ uint32_t order_bucket(int32_t v, int32_t lo, int32_t hi)
{
    const uint64_t span = (uint64_t)((int64_t)hi - (int64_t)lo) + 1u;
    return (uint32_t)(((uint64_t)((int64_t)v - (int64_t)lo) * kOrderBuckets) / span);
}

// tab: [0] min, [1] max, [2 ..] buckets
__global__ void __launch_bounds__(256) order_minmax(SParams p, int32_t *tab)
{
    int32_t lo = INT32_MAX, hi = INT32_MIN;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < p.n; i += (uint64_t)gridDim.x * 256u) {
        const int32_t v = sched_input(p, i);
        lo = v < lo ? v : lo;
        hi = v > hi ? v : hi;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const int32_t a = __shfl_xor(lo, o, 64), b = __shfl_xor(hi, o, 64);
        lo = a < lo ? a : lo;
        hi = b > hi ? b : hi;
    }
    if ((threadIdx.x & 63u) == 0) {
        atomicMin(&tab[0], lo);
        atomicMax(&tab[1], hi);
    }
}

__global__ void __launch_bounds__(256) order_hist(SParams p, int32_t *tab)
{
    __shared__ uint32_t h[kOrderBuckets];
    for (uint32_t b = threadIdx.x; b < kOrderBuckets; b += 256u) h[b] = 0u;
    __syncthreads();
    const int32_t lo = tab[0], hi = tab[1];
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < p.n; i += (uint64_t)gridDim.x * 256u)
        atomicAdd(&h[order_bucket(sched_input(p, i), lo, hi)], 1u);
    __syncthreads();
    uint32_t *g = (uint32_t *)(tab + 2);
    for (uint32_t b = threadIdx.x; b < kOrderBuckets; b += 256u)
        if (h[b]) atomicAdd(&g[b], h[b]);
}

// exclusive prefix sum of the buckets, in place (one block of 1024)
__global__ void __launch_bounds__(1024) order_scan(int32_t *tab)
{
    __shared__ uint32_t part[1024];
    uint32_t *g = (uint32_t *)(tab + 2);
    const uint32_t t = threadIdx.x, per = kOrderBuckets / 1024u;
    uint32_t sum = 0;
    for (uint32_t k = 0; k < per; ++k) sum += g[t * per + k];
    part[t] = sum;
    __syncthreads();
    for (uint32_t o = 1; o < 1024u; o <<= 1) {
        const uint32_t v = t >= o ? part[t - o] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint32_t run = part[t] - sum;
    for (uint32_t k = 0; k < per; ++k) {
        const uint32_t c = g[t * per + k];
        g[t * per + k] = run;
        run += c;
    }
}

__global__ void __launch_bounds__(256) order_scatter(SParams p, int32_t *tab, uint32_t *order)
{
    const int32_t lo = tab[0], hi = tab[1];
    uint32_t *g = (uint32_t *)(tab + 2);
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < p.n; i += (uint64_t)gridDim.x * 256u)
        order[atomicAdd(&g[order_bucket(sched_input(p, i), lo, hi)], 1u)] = (uint32_t)i;
}

__global__ void __launch_bounds__(kBlock) gen_inputs(uint64_t seed, uint32_t kind, uint32_t mask,
                                                     uint64_t offset, uint64_t n, int32_t *out)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        out[i] = gen_value(seed, kind, mask, offset + i);
}

// Dependency-free integer adds: 8 independent chains x 8 adds per iteration.
__global__ void __launch_bounds__(kBlock) valu_probe(int iters, uint32_t *sink)
{
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
             a6 = a0 + 6, a7 = a0 + 7;
    const uint32_t c = blockIdx.x | 1u;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            asm volatile("v_add_u32 %0, %0, %8\n\t"
                         "v_add_u32 %1, %1, %8\n\t"
                         "v_add_u32 %2, %2, %8\n\t"
                         "v_add_u32 %3, %3, %8\n\t"
                         "v_add_u32 %4, %4, %8\n\t"
                         "v_add_u32 %5, %5, %8\n\t"
                         "v_add_u32 %6, %6, %8\n\t"
                         "v_add_u32 %7, %7, %8"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                         : "v"(c));
        }
    }
    if ((a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7) == 0x9E3779B9u) sink[0] = 1;
}

// ------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------
struct SchedDev {
    DOp *d_code = nullptr;
    uint32_t block = 0, slots = 0;
    uint32_t *d_entry = nullptr;
    uint32_t *d_jtab = nullptr;
    int32_t *d_slots = nullptr;
    size_t slots_bytes = 0;
    uint32_t *d_order = nullptr; // machine shape: input order of a launch (order_* kernels)
    size_t order_cap = 0;
    int32_t *d_ordtab = nullptr; // min, max, buckets
};

// Tier 3: the schedule compiled to a native kernel (tis_jit.h).
// Grid of the tile-sorted machine kernel for networks with stack slots in
// HBM, measured (launch_jit_locked): the first launches at a batch size run
// the resident grid and two smaller ones (3/4, 1/2 of its blocks), each
// bracketed by events; the first launch after all three have completed
// (hipEventQuery, never waiting) keeps the fastest.  Slot-heavy kernels split
// on it: t1_two_stacks (1 KiB of stores per lane) runs 233 -> 192 us at 3/4
// of the blocks, t2_dyn_depth (pushes read back) 119 -> 138 us
// (profiles/r08_grid_tune_ab.txt).  Results do not depend on the grid.
struct GridTune {
    uint64_t n = 0;          // batch size the state is for (another size starts over)
    int phase = 0;           // 0..2: candidate `phase` launched next; 3: deciding; 4: decided
    int cand[3] = {0, 0, 0}; // blocks: 3/4, 1/2, all of the resident grid (cold launch first)
    int chosen = 0;
    float ms[3] = {0, 0, 0};
    hipEvent_t ev[6] = {};
};

struct JitDev {
    hipModule_t mod = nullptr;
    hipFunction_t fn = nullptr;
    int per_cu = 0;
    int last_blocks = 0; // grid of the last launch (a batch smaller than the resident grid, or GridTune's)
    GridTune tune[4];    // by batch size, the oldest replaced
    int tune_next = 0;
    int tune_last = -1;  // entry of the last tuned launch
};

struct JitState {
    bool tried = false, ok = false;
    std::string why;          // reason the native tier is unavailable
    std::vector<char> code;   // gfx950 code object
    double compile_s = 0;
    size_t src_bytes = 0;
    uint64_t src_hash = 0;    // FNV-1a of the module source: which kernel a profile describes
    JitShape shape = JIT_STREAM;
    uint64_t max_steps = UINT64_MAX; // stream shape: launches need budget > max_steps
    bool heavy = false;              // stream shape, one lane per thread (kStreamKernelHeavy)
    bool lds = false;                // heavy kernel with all its stack slots in LDS (no HBM slots)
    uint32_t lds_n = 0;              // heavy kernel: slots per lane in LDS (the rest in HBM)
    std::string rtc;                 // compiler of the module: linked / ns / linked-other
    uint32_t pool = 0;               // machine shape: lane-pool slots per wave (kMachinePoolKernel)
    int block = kJitBlock;
    JitDev dev[kMaxDevices];
};

// One way to run a heavy stream network with stack slots (tune_lds_auto):
// its schedule, LDS bytes of slots per wave, micro-op bound, and the waves
// per SIMD it is meant for (0: none checked).
struct StackPlan {
    SchedProgram prog;
    size_t lds_bytes = 0;
    size_t max_dops = 0;
    uint32_t waves = 0;
};

// A compiled schedule for one (stack_cap, stop_on_output) pair.
struct SchedCache {
    uint32_t cap = 0;
    bool soo = false;
    bool ok = false;
    bool tile = false; // default lane scheduling (sched_default_tile)
    bool lds_set = false;   // tune_soft_regs chose the heavy kernel's LDS budget ...
    size_t lds_bytes = 0;   // ... this many bytes of slots per wave (0: slots in HBM)
    size_t max_dops = 0;    // ... and a larger micro-op bound for its unrolled register entries (0: the knob's)
    uint32_t want_waves = 0;  // waves per SIMD the schedule is for: its module's registers are checked (0: none)
    std::vector<StackPlan> alts; // the next plans to try when that check fails (tune_lds_auto)
    std::string occ_note;     // what the check found (mk_net_plan occupancy=)
    std::string why;
    SchedProgram prog;  // the schedule the native tier compiles (a more_waves plan, or the default)
    // Tier 2's schedule while the native tier tries a more_waves plan: the
    // default plan (its register file lives in LDS, so the plans' hundreds of
    // registers would leave tier 2 one 64-lane block per CU).  Null: prog.
    std::unique_ptr<SchedProgram> t2;
    SchedDev dev[kMaxDevices];
    JitState jit;
};

// The schedule tier 2 (and the interpreter's superblock-count test) uses.
const SchedProgram &tier2_prog(const SchedCache *sc) { return sc->t2 ? *sc->t2 : sc->prog; }

struct DevCtx {
    bool ready = false;
    Insn *d_code = nullptr;
    int cus = 0;
    int32_t *d_spill = nullptr;
    size_t spill_bytes = 0;
    // host-API staging (mk_compute_batch): device buffers for one call's
    // share, and a pinned host mirror while that share fits one chunk
    void *d_stage = nullptr;
    void *h_stage = nullptr;
    size_t stage_bytes = 0;
    unsigned long long *d_partials = nullptr; // per-wave counters
    size_t partials_bytes = 0;
    hipStream_t stream = nullptr;
    // The handle's per-device scratch (stack slots, spill rows, counters,
    // staging) is shared by every stream that launches on it: the host API
    // uses `stream`, the device API the caller's.  Work is ordered across a
    // change of stream (order_on): the new stream waits for an event
    // recorded on the previous one.
    hipStream_t last = nullptr;
    bool used = false;
    hipEvent_t ev = nullptr;
};

// Native modules loaded once per (device, code object) and never unloaded
// with MK_JIT_KEEP_MODULES=1 (diagnostics); by default each network unloads
// its own.  Networks and sessions whose code objects are equal share one
// kept module.
inline bool keep_module(const std::string &)
{
    static const bool k = [] {
        const char *s = std::getenv("MK_JIT_KEEP_MODULES");
        return s && *s == '1';
    }();
    return k;
}

struct KeptModule {
    int dev;
    std::vector<char> code; // the image stays alive with its module
    hipModule_t mod;
};

// hipModuleLoadData, or the kept module of an equal code object.  Caller
// has the device current.
inline hipError_t load_module(int dev, const std::vector<char> &code, const std::string &from, hipModule_t *mod)
{
    if (!keep_module(from)) return hipModuleLoadData(mod, code.data());
    static std::mutex mu;
    static auto *kept = new std::deque<KeptModule>(); // never freed
    std::lock_guard<std::mutex> g(mu);
    for (const KeptModule &k : *kept)
        if (k.dev == dev && k.code == code) {
            *mod = k.mod;
            return hipSuccess;
        }
    kept->push_back(KeptModule{dev, code, nullptr});
    const hipError_t e = hipModuleLoadData(&kept->back().mod, kept->back().code.data());
    if (e != hipSuccess) {
        kept->pop_back();
        return e;
    }
    *mod = kept->back().mod;
    return hipSuccess;
}

inline void release_module(hipModule_t mod, const std::string &from)
{
    if (mod && !keep_module(from)) (void)hipModuleUnload(mod);
}

} // namespace mk

struct mk_net {
    mk::Network net;
    std::mutex mu;      // serialises host-API calls, compilation and device-context setup
    mk::DevCtx dev[mk::kMaxDevices];
    std::vector<std::unique_ptr<mk::SchedCache>> sched;
    mk::JitLimits jit_lim = mk::JitLimits::from_env(); // knob snapshot at load (tis_jit.h)
    uint64_t host_chunk = 0;                           // mk_compute_batch chunk (inputs)
    ~mk_net()
    {
        int prev = 0;
        (void)hipGetDevice(&prev);
        for (int d = 0; d < mk::kMaxDevices; d++) {
            mk::DevCtx &c = dev[d];
            if (!c.ready) continue;
            (void)hipSetDevice(d);
            if (c.stream) (void)hipStreamSynchronize(c.stream);
            (void)hipFree(c.d_code);
            (void)hipFree(c.d_spill);
            (void)hipFree(c.d_stage);
            (void)hipHostFree(c.h_stage);
            (void)hipFree(c.d_partials);
            for (auto &sc : sched) {
                (void)hipFree(sc->dev[d].d_code);
                (void)hipFree(sc->dev[d].d_entry);
                (void)hipFree(sc->dev[d].d_jtab);
                (void)hipFree(sc->dev[d].d_slots);
                (void)hipFree(sc->dev[d].d_order);
                (void)hipFree(sc->dev[d].d_ordtab);
                mk::release_module(sc->jit.dev[d].mod, sc->jit.rtc);
                for (const mk::GridTune &t : sc->jit.dev[d].tune)
                    for (hipEvent_t e : t.ev)
                        if (e) (void)hipEventDestroy(e);
            }
            if (c.stream) (void)hipStreamDestroy(c.stream);
            if (c.ev) (void)hipEventDestroy(c.ev);
        }
        (void)hipSetDevice(prev);
    }
};

namespace mk {
namespace {

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int d)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != d) (void)hipSetDevice(d);
    }
    ~DeviceGuard()
    {
        int cur = -1;
        (void)hipGetDevice(&cur);
        if (prev >= 0 && cur != prev) (void)hipSetDevice(prev);
    }
};

int device_count()
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

// Caller holds net->mu.
int ensure_device(mk_net *h, int d)
{
    DevCtx &c = h->dev[d];
    if (c.ready) return MK_OK;
    DeviceGuard g(d);
    const size_t bytes = h->net.code.size() * sizeof(Insn);
    if (hipMalloc(&c.d_code, bytes) != hipSuccess) return MK_ENOMEM;
    if (hipMemcpy(c.d_code, h->net.code.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) return MK_EDEVICE;
    if (hipDeviceGetAttribute(&c.cus, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess) return MK_EDEVICE;
    if (hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking) != hipSuccess) return MK_EDEVICE;
    if (hipEventCreateWithFlags(&c.ev, hipEventDisableTiming) != hipSuccess) return MK_EDEVICE;
    c.ready = true;
    return MK_OK;
}

// Caller holds h->mu, device d current.  Work about to be enqueued on `s`
// that touches the handle's scratch on this device: if the previous such
// work went to another stream, `s` first waits for it.  Free when the
// stream does not change (the bench's and the master's steady state).
int order_on(DevCtx &c, hipStream_t s)
{
    if (c.used && c.last != s) {
        if (hipEventRecord(c.ev, c.last) != hipSuccess || hipStreamWaitEvent(s, c.ev, 0) != hipSuccess)
            return MK_EDEVICE;
    }
    c.used = true;
    c.last = s;
    return MK_OK;
}

template <int NMAX>
void *kernel_ptr() { return reinterpret_cast<void *>(&tis_exec<NMAX>); }

void *pick_kernel(int nprog)
{
    if (nprog <= 1) return kernel_ptr<1>();
    if (nprog <= 2) return kernel_ptr<2>();
    if (nprog <= 4) return kernel_ptr<4>();
    if (nprog <= 8) return kernel_ptr<8>();
    return kernel_ptr<16>();
}

struct Launch {
    void *fn;
    int blocks;
    size_t lds;
    uint32_t ring;
};

// Shape the launch: LDS ring depth, dynamic LDS bytes, resident grid.
int plan_launch(const Network &net, const DevCtx &c, size_t n, uint32_t stack_cap, Launch &L)
{
    L.fn = pick_kernel(net.nprog);
    uint32_t ring = 0;
    int stack_rows = 0;
    if (net.uses_stacks) {
        // Keep >= 2 blocks per CU: <= 80 KiB of LDS per 256-lane block.
        ring = 16;
        while (ring > 1 && (size_t)(net.nprog * 4 + net.nstack * (1 + ring)) * kBlock * 4 > 80 * 1024) ring >>= 1;
        stack_rows = net.nstack;
    }
    const size_t lds = (size_t)(net.nprog * 4 + stack_rows * (1 + ring)) * kBlock * 4;
    if (lds > 160 * 1024) return MK_ELIMIT;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, L.fn, kBlock, lds) != hipSuccess || per_cu < 1)
        per_cu = 1;
    const uint64_t want = (n + kBlock - 1) / kBlock;
    const uint64_t resident = (uint64_t)per_cu * (uint64_t)std::max(c.cus, 1);
    L.blocks = (int)std::max<uint64_t>(1, std::min<uint64_t>(want, resident));
    L.lds = lds;
    L.ring = ring;
    (void)stack_cap;
    return MK_OK;
}

void resolve_opts(const mk_opts *o, uint32_t &budget, uint32_t &cap, uint32_t &flags)
{
    budget = (o && o->budget) ? o->budget : (1u << 20);
    if (budget > 0xFFFFFF00u) budget = 0xFFFFFF00u; // steps (u32) may overshoot by < 16
    cap = (o && o->stack_cap) ? o->stack_cap : 1024u;
    flags = o ? o->flags : 0u;
}

// Default lane scheduling: tiles.  Measured on MI355X (profiles/r01_modes.txt)
// tiles beat refill on every configuration, including the variable-length
// C5 countdown (vector I/O and one shared superblock walk per tile outweigh
// the idle slots of finished lanes).
bool sched_default_tile(const SchedProgram &) { return true; }

// Waves per CU the heavy kernel's LDS-resident slots allow (capped at 4, one
// per SIMD); 0 when its slots stay in HBM.
uint32_t lds_waves(const SchedProgram &P, const JitLimits &lim)
{
    if (!jit_slots_in_lds(P.nslots, true, lim)) return 0;
    // LDS allocation granule: measured, 207 slots (52,992 B) fit three waves per
    // CU and 212 (54,272 B) do not (r02af), so a 2 KiB granule is assumed
    const uint64_t bytes = ((uint64_t)P.nslots * 256u + 2047u) / 2048u * 2048u;
    return std::min<uint32_t>(4u, (uint32_t)((160u * 1024u) / bytes));
}

// A network that runs on the heavy stream kernel with its stack slots in
// LDS is latency-bound when they allow fewer than one wave per SIMD (C4
// D=256: 233 slots, 58 KB, two waves per CU: 0.61 ms).  Keeping more stack
// entries in registers (SchedLimits::soft_regs) leaves fewer slots: the
// smallest register count that reaches the most waves (up to four) wins --
// C4 D=256 at 50 registers: 207 slots, three waves, 0.38 ms (r02ae; D=64,
// 15 waves already, is fastest at the default 24; 212 slots stayed at two
// waves, 0.56 ms, r02af).  Heavy stream networks whose slots stay in HBM
// take up to 64 registers (fewer slot bytes per lane; see below).
// MK_JIT_TUNE_REGS=0 keeps the default.
// Whether the native tier takes P as a heavy stream lane.
bool heavy_stream(const SchedProgram &P, const JitLimits &jl)
{
    std::string src, why;
    JitShape shape = JIT_STREAM;
    bool heavy = false;
    return jit_lane_source(P, jl, src, why, &shape, nullptr, &heavy) && shape == JIT_STREAM && heavy;
}

// More waves per SIMD for heavy LDS networks (round 5).  At one wave per
// SIMD a gfx950 wave issues a VALU op only every ~8.8 cycles; C4 D=256's
// default kernel (64 registers, 160 of 193 slots in LDS, one wave per SIMD)
// spent its time there (profiles/r06b_pmc_stall_c4d256_c5.txt).  Keeping more
// stack entries in registers (SchedLimits::soft_regs) leaves fewer slots, and
// W waves per SIMD leave each wave 160 KiB / 4W of LDS.  For W = 8 and then
// 2, a register count up to kStackRegs that puts every slot in that share
// makes a plan, with a micro-op bound of kStackDops for the unrolled
// register entries.  Registers are the risk: a program whose register-held
// entries stay live needs more VGPRs than W waves allow, so jit_compile
// checks the compiled module (vgprs, agprs, scratch) against W and falls back
// to the next plan, and last to the one-wave default (which is not checked).
// Measured on MI355X (r06f/r06g, C4 D=256, 512K lanes): the default 159.8 us;
// two waves, 80 slots in LDS, 128 / 144 / 152 / 176 registers (49 / 33 / 25 /
// 1 slots left in HBM) 126.5 / 80.3 / 69.5 / 55.0 us; three waves (208
// registers, 48 slots in LDS) 13.9 us.  With the stack entries in registers
// LLVM sees the pushed values and folds the pipeline's pop chains, so the
// stack traffic per PUSH/POP falls with the registers (bench.py reports it,
// `stack.stack_ops_executed_per_push_pop`).
constexpr uint32_t kStackRegs = 256;
constexpr size_t kStackDops = 16384;

std::vector<StackPlan> more_waves(mk_net *h, SchedCache *sc, const SchedLimits &lim0, uint32_t regs0, uint32_t slots0)
{
    std::vector<StackPlan> out;
    const JitLimits &jl = h->jit_lim;
    if (!jl.lds_slot_bytes) return out;
    JitLimits jl2 = jl;
    jl2.max_dops = std::max(jl.max_dops, kStackDops);
    // Each added register takes about one slot (an entry of the deepest
    // stack window): start at the count that predicts a fit and step up.
    // compile_schedule takes seconds on deep pipelines, so few probes.
    for (uint32_t waves : {8u, 2u}) {
        const uint64_t cap = std::min<uint64_t>(jl.lds_slot_bytes, (160u * 1024u) / (4u * waves) / 2048u * 2048u);
        const uint32_t k = (uint32_t)(cap / 256u); // slots of a wave's LDS share
        if (slots0 <= k) continue;
        for (uint32_t r = regs0 + (slots0 - k), probes = 0; r <= kStackRegs && probes < 4; r += 4u, ++probes) {
            SchedLimits l = lim0;
            l.soft_regs = r;
            l.max_regs = std::max(l.max_regs, r + 24u);
            StackPlan sp;
            std::string w;
            if (!compile_schedule(h->net, sc->cap, sc->soo, l, sp.prog, w) || !heavy_stream(sp.prog, jl2)) break;
            if (sp.prog.nslots > k) continue;
            sp.lds_bytes = (size_t)cap;
            sp.max_dops = jl2.max_dops;
            sp.waves = waves;
            out.push_back(std::move(sp));
            break;
        }
    }
    return out;
}

// Installs a plan (a tuning choice, or the next after a failed check).
void use_plan(SchedCache *sc, StackPlan &&sp)
{
    if (!sp.waves) sc->t2.reset(); // the default plan: tier 2's own (tier2_prog)
    sc->prog = std::move(sp.prog);
    sc->lds_set = true;
    sc->lds_bytes = sp.lds_bytes;
    sc->max_dops = sp.max_dops;
    sc->want_waves = sp.waves;
}

// Default policy for heavy stream networks (JitLimits::lds_auto): waves per
// CU first, then as many slots in LDS as those waves leave room for.
//   * slots that fit LDS at four waves per CU at the default registers: keep
//     them there (C4 D=64: 41 slots, 15 waves);
//   * else take the most registers up to 64 the native tier accepts (fewer
//     slots; r02ap) and the most waves w in 4, 3, 2 whose LDS share (160,
//     208, 320 slots in 2 KiB granules) holds all the slots or at least
//     lds_split percent of them (the rest in HBM); none: slots in HBM.
// Measured (r02av, 256K-512K lanes): C4 D=256 four waves, 160 of 193 slots
// in LDS 325 us (three waves, all 208 in LDS: 386); D=320 three waves, 208
// of 257: 302 us (two waves, all in LDS: 497); D=400 two waves, 320 of 337:
// 571 us (three waves, 208: 661); D=480 two waves, 320 of 417: 655 us (HBM:
// 1,048); at 64% or less in LDS HBM alone is as fast or faster (r02au).
void tune_lds_auto(mk_net *h, SchedCache *sc, const SchedLimits &lim0)
{
    const JitLimits &jl = h->jit_lim;
    auto bytes = [&](uint32_t n) { return ((uint64_t)n * 256u + 2047u) / 2048u * 2048u; };
    if (!heavy_stream(sc->prog, jl)) return;
    if (jl.lds_slot_bytes && bytes(sc->prog.nslots) * 4u <= 160u * 1024u) {
        // the knob's budget holds them at four waves per CU (C4 D=64: 41
        // slots, 15 waves per CU): more waves per SIMD when more registers
        // shrink the slots to their share (more_waves), else as they are
        std::vector<StackPlan> more = more_waves(h, sc, lim0, sc->prog.nregs, sc->prog.nslots);
        if (more.empty()) return;
        StackPlan def;
        def.prog = sc->prog;
        def.lds_bytes = jl.lds_slot_bytes;
        for (size_t k = 1; k < more.size(); ++k) sc->alts.push_back(std::move(more[k]));
        sc->t2 = std::make_unique<SchedProgram>(def.prog); // tier 2 keeps the default plan
        sc->alts.push_back(std::move(def));
        use_plan(sc, std::move(more[0]));
        return;
    }
    SchedProgram best = sc->prog;
    for (uint32_t r = 64u; r > lim0.soft_regs; r -= 8u) {
        SchedLimits l = lim0;
        l.soft_regs = r;
        SchedProgram P;
        std::string w;
        if (compile_schedule(h->net, sc->cap, sc->soo, l, P, w) && heavy_stream(P, jl)) {
            best = std::move(P);
            break;
        }
    }
    size_t budget = 0;
    if (jl.lds_slot_bytes)
        for (uint32_t w = 4; w >= 2; --w) {
            const uint64_t cap = std::min<uint64_t>(jl.lds_slot_bytes, (160u * 1024u) / w / 2048u * 2048u);
            const uint64_t k = cap / 256u; // slots of one wave in LDS
            if (bytes(best.nslots) <= cap || (jl.lds_split && k * 100u >= (uint64_t)best.nslots * jl.lds_split)) {
                budget = (size_t)cap;
                break;
            }
        }
    std::vector<StackPlan> more = more_waves(h, sc, lim0, best.nregs, best.nslots);
    StackPlan def;
    def.prog = std::move(best);
    def.lds_bytes = budget;
    if (more.empty()) {
        use_plan(sc, std::move(def));
        return;
    }
    for (size_t k = 1; k < more.size(); ++k) sc->alts.push_back(std::move(more[k]));
    sc->t2 = std::make_unique<SchedProgram>(def.prog); // tier 2 keeps the default plan
    sc->alts.push_back(std::move(def));
    use_plan(sc, std::move(more[0]));
}

// MK_JIT_LDS_SLOTS set: registers for the fixed LDS budget (see above).
void tune_soft_regs_fixed(mk_net *h, SchedCache *sc, const SchedLimits &lim0)
{
    const JitLimits &jl = h->jit_lim;
    const uint32_t w0 = lds_waves(sc->prog, jl);
    if (w0 >= 4) return;
    // waves of the program compiled with r registers, 0 unless the native
    // tier takes it as a heavy stream lane with LDS slots
    auto waves = [&](uint32_t r, SchedProgram &P) -> uint32_t {
        SchedLimits l = lim0;
        l.soft_regs = r;
        std::string w, src;
        JitShape shape = JIT_STREAM;
        bool heavy = false;
        if (!compile_schedule(h->net, sc->cap, sc->soo, l, P, w)) return 0;
        if (!jit_lane_source(P, jl, src, w, &shape, nullptr, &heavy) || shape != JIT_STREAM || !heavy) return 0;
        return lds_waves(P, jl);
    };
    {
        std::string src, why;
        JitShape shape = JIT_STREAM;
        bool heavy = false;
        if (!jit_lane_source(sc->prog, jl, src, why, &shape, nullptr, &heavy) || shape != JIT_STREAM || !heavy)
            return; // not a heavy stream lane
    }
    if (w0 == 0) {
        // Slots in HBM: fewer slot bytes per lane with more entries in
        // registers (r02ap, 256K lanes: C4 D=400 950 -> 810 us at 64
        // registers, D=640 1,684 -> 1,473, D=1024 2,922 -> 2,752): the most
        // registers up to 64 that the native tier still takes.
        for (uint32_t r = 64u; r > lim0.soft_regs; r -= 8u) {
            SchedLimits l = lim0;
            l.soft_regs = r;
            SchedProgram P;
            std::string w, src;
            JitShape shape = JIT_STREAM;
            bool heavy = false;
            if (compile_schedule(h->net, sc->cap, sc->soo, l, P, w) &&
                jit_lane_source(P, jl, src, w, &shape, nullptr, &heavy) && shape == JIT_STREAM && heavy) {
                sc->prog = std::move(P);
                return;
            }
        }
        return;
    }
    // coarse scan for the most waves, then the fewest registers that reach them
    uint32_t best_w = w0, best_r = lim0.soft_regs, prev_r = lim0.soft_regs;
    for (uint32_t r = lim0.soft_regs + 8u; r + 8u <= lim0.max_regs && best_w < 4u; r += 8u) {
        SchedProgram P;
        const uint32_t w = waves(r, P);
        if (!w) break;
        if (w > best_w) best_w = w, best_r = r;
        if (best_r != r) prev_r = r;
        // about one slot fewer per register: stop when the next step is out of reach
        const uint32_t next = (160u * 1024u / 2048u) / (w + 1u) * 8u;
        if (w < 4u && P.nslots > next && P.nslots - next > lim0.max_regs - 8u - r) break;
    }
    if (best_w == w0) return;
    uint32_t lo = prev_r + 1u, top = best_r;
    while (lo < top) {
        const uint32_t mid = (lo + top) / 2u;
        SchedProgram P;
        if (waves(mid, P) >= best_w) top = mid;
        else lo = mid + 1u;
    }
    SchedProgram P;
    if (waves(top, P) >= best_w) sc->prog = std::move(P);
}

void tune_soft_regs(mk_net *h, SchedCache *sc, const SchedLimits &lim0)
{
    const JitLimits &jl = h->jit_lim;
    if (!jl.tune_regs || jl.disabled || !sc->prog.nslots) return;
    if (jl.lds_auto) {
        tune_lds_auto(h, sc, lim0);
        return;
    }
    tune_soft_regs_fixed(h, sc, lim0);
}

// Caller holds h->mu.  Compiles the schedule for (cap, soo) once.
SchedCache *get_sched(mk_net *h, uint32_t cap, bool soo)
{
    for (auto &sc : h->sched)
        if (sc->cap == cap && sc->soo == soo) return sc.get();
    auto sc = std::make_unique<SchedCache>();
    sc->cap = cap;
    sc->soo = soo;
    SchedLimits lim;
    sc->ok = compile_schedule(h->net, cap, soo, lim, sc->prog, sc->why);
    if (sc->ok) tune_soft_regs(h, sc.get(), lim);
    sc->tile = sc->ok && sched_default_tile(sc->prog);
    h->sched.push_back(std::move(sc));
    return h->sched.back().get();
}

// Launch geometry of the tier-2 kernel for a program with `nregs` registers:
// block size B and K input slots per thread, LDS nregs*K*B*8 <= 40 KiB.
void sched_geometry(uint32_t nregs, uint32_t &B, uint32_t &K)
{
    const size_t r = (size_t)nregs + 1; // + scratch register
    B = 256;
    while (B > 64 && r * B * 8 > 40 * 1024) B >>= 1;
    K = 4;
    while (K > 1 && r * K * B * 8 > 40 * 1024) K >>= 1;
}

template <int K, int B>
void *sched_kernel_t(bool tile)
{
    return tile ? reinterpret_cast<void *>(&tis_sched_tile<K, B>) : reinterpret_cast<void *>(&tis_sched_exec<K, B>);
}

void *sched_kernel(int K, int B, bool tile)
{
    if (B == 256 && K == 4) return sched_kernel_t<4, 256>(tile);
    if (B == 256 && K == 2) return sched_kernel_t<2, 256>(tile);
    if (B == 256 && K == 1) return sched_kernel_t<1, 256>(tile);
    if (B == 128 && K == 1) return sched_kernel_t<1, 128>(tile);
    if (B == 64 && K == 1) return sched_kernel_t<1, 64>(tile);
    return nullptr;
}


// Caller holds h->mu.
int ensure_sched_device(SchedCache *sc, int d)
{
    SchedDev &sd = sc->dev[d];
    if (sd.d_code) return MK_OK;
    DeviceGuard g(d);
    const SchedProgram &P = tier2_prog(sc);
    sched_geometry(P.nregs, sd.block, sd.slots);
    std::vector<uint32_t> entry;
    const std::vector<DOp> code = assemble_device(P, sd.block * sd.slots * 8, entry);
    const size_t cb = code.size() * sizeof(DOp), eb = entry.size() * 4, jb = std::max<size_t>(P.jtab.size(), 1) * 4;
    if (hipMalloc(&sd.d_code, cb) != hipSuccess || hipMalloc(&sd.d_entry, eb) != hipSuccess ||
        hipMalloc(&sd.d_jtab, jb) != hipSuccess)
        return MK_ENOMEM;
    if (hipMemcpy(sd.d_code, code.data(), cb, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(sd.d_entry, entry.data(), eb, hipMemcpyHostToDevice) != hipSuccess ||
        (!P.jtab.empty() && hipMemcpy(sd.d_jtab, P.jtab.data(), P.jtab.size() * 4, hipMemcpyHostToDevice) != hipSuccess))
        return MK_EDEVICE;
    return MK_OK;
}

// Caller holds h->mu.  Per-wave counter buffer for `lanes` resident lanes.
// The per-wave counter rows are allocated once per device context for the
// largest resident grid (2048 threads per CU) and zeroed; kernels add into
// them and stats_reduce folds and clears them, so counts of launches that
// defer their stats (MK_FLAG_DEFER_STATS) accumulate until the next fold.
int ensure_partials(DevCtx &c, uint64_t lanes)
{
    if (!c.d_partials) {
        const size_t rows = (size_t)std::max(c.cus, 1) * 32;
        const size_t bytes = rows * 8 * sizeof(unsigned long long);
        if (hipMalloc(&c.d_partials, bytes) != hipSuccess) return MK_ENOMEM;
        if (hipMemset(c.d_partials, 0, bytes) != hipSuccess) return MK_EDEVICE;
        c.partials_bytes = bytes;
    }
    return (lanes + 63) / 64 <= c.partials_bytes / 64 ? MK_OK : MK_ELIMIT; // one 64-byte row per wave
}

int launch_stats_reduce(DevCtx &c, uint64_t *d_stats, hipStream_t stream)
{
    const uint32_t nrows = (uint32_t)(c.partials_bytes / 64);
    hipLaunchKernelGGL(stats_reduce, dim3((nrows + 255) / 256), dim3(256), 0, stream, c.d_partials, nrows,
                       reinterpret_cast<unsigned long long *>(d_stats));
    return hipGetLastError() == hipSuccess ? MK_OK : MK_EDEVICE;
}

// Counters are gathered when the caller passes stats or defers them; folded
// into d_stats right after the launch unless deferred.
bool counting(const uint64_t *d_stats, uint32_t flags) { return d_stats || (flags & MK_FLAG_DEFER_STATS); }
bool fold_now(const uint64_t *d_stats, uint32_t flags) { return d_stats && !(flags & MK_FLAG_DEFER_STATS); }

// Caller holds h->mu.  Tier-2 launch; asynchronous on `stream`.
int launch_sched_locked(mk_net *h, SchedCache *sc, int d, const mk_input *in, size_t n, int32_t *d_out,
                        uint8_t *d_status, uint32_t *d_steps, uint64_t *d_stats, uint32_t budget, uint32_t flags,
                        hipStream_t stream)
{
    int rc = ensure_sched_device(sc, d);
    if (rc) return rc;
    DevCtx &c = h->dev[d];
    SchedDev &sd = sc->dev[d];
    const SchedProgram &P = tier2_prog(sc);
    DeviceGuard g(d);
    // LDS register file [nregs][K][B] x 8 B; block size and slot count are
    // fixed by the assembly (sched_geometry).
    const int B = (int)sd.block, K = (int)sd.slots;
    const size_t lds = (size_t)(P.nregs + 1) * K * B * 8; // + one scratch register
    if (lds > 160 * 1024) return MK_ELIMIT;
    const bool tile = (flags & MK_FLAG_TILE) ? true : (flags & MK_FLAG_REFILL) ? false : sc->tile;
    void *fn = sched_kernel(K, B, tile);
    if (!fn) return MK_ELIMIT;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, B, lds) != hipSuccess || per_cu < 1) per_cu = 1;
    const uint64_t want = (n + (uint64_t)B * K - 1) / ((uint64_t)B * K); // tiles
    const uint64_t resident = (uint64_t)per_cu * (uint64_t)std::max(c.cus, 1);
    const int blocks = (int)std::max<uint64_t>(1, std::min<uint64_t>(want, resident));
    const uint64_t lanes = (uint64_t)blocks * B;
    const uint64_t vlanes = lanes * (uint64_t)K;
    if (P.nslots) {
        const size_t need = (size_t)(P.nslots + 1) * vlanes * sizeof(int32_t); // + scratch row
        if (need > sd.slots_bytes) {
            if (sd.d_slots) {
                (void)hipDeviceSynchronize();
                (void)hipFree(sd.d_slots);
                sd.d_slots = nullptr;
                sd.slots_bytes = 0;
            }
            if (hipMalloc(&sd.d_slots, need) != hipSuccess) return MK_ENOMEM;
            sd.slots_bytes = need;
        }
    }
    SParams p{};
    p.in_kind = in->kind;
    p.gen_kind = in->gen_kind;
    p.in_data = in->data;
    p.seed = in->seed;
    p.offset = in->offset;
    p.gen_mask = in->gen_mask;
    p.budget = budget;
    p.n = n;
    p.out = d_out;
    p.status = d_status;
    p.steps = d_steps;
    if (counting(d_stats, flags) && (rc = ensure_partials(c, lanes))) return rc;
    p.partials = counting(d_stats, flags) ? c.d_partials : nullptr;
    p.slots = sd.d_slots;
    p.lanes = lanes;
    p.vlanes = vlanes;
    p.in_off = P.in_reg * (uint32_t)(K * B * 8);
    p.scratch_off = P.nregs * (uint32_t)(K * B * 8);
    p.scratch_slot = P.nslots;
    const uintptr_t va = 4u * (uintptr_t)K; // K x int32 vector
    p.io_vec = in->kind == MK_IN_I32 && (uintptr_t)in->data % va == 0 && (uintptr_t)d_out % va == 0 &&
               (uintptr_t)d_status % (uintptr_t)K == 0 && (uintptr_t)d_steps % va == 0;
    const DOp *code = sd.d_code;
    const uint32_t *entry = sd.d_entry, *jtab = sd.d_jtab;
    void *args[] = {(void *)&code, (void *)&entry, (void *)&jtab, (void *)&p};
    if (hipLaunchKernel(fn, dim3(blocks), dim3(B), args, lds, stream) != hipSuccess) return MK_EDEVICE;
    return fold_now(d_stats, flags) ? launch_stats_reduce(c, d_stats, stream) : MK_OK;
}

// ---- tier 3: native kernel per schedule (tis_jit.h) ------------------------
// One hiprtc compilation, run on a compile thread so that the caller can
// give up after lim.max_compile_s: the job owns its inputs and outputs
// (shared), so a compile the caller abandoned finishes in the background and
// is discarded.
struct HiprtcJob {
    std::string src;
    std::vector<std::string> env; // the caller's environment, copied on the caller's thread (rtc_compile)
    std::mutex mu;
    std::condition_variable cv;
    bool done = false, ok = false;
    bool abandoned = false; // the caller gave up (under mu)
    std::string why;
    std::vector<char> code;
};

// Compiles still running on detached threads: the library's teardown waits
// for them (a thread inside comgr while static destructors run would crash).
// Diagnostics (MK_SEGV_TRACE=1): a fatal signal in any thread prints that
// thread's native backtrace (library+offset per frame) before the handler
// that was installed before it (Python's faulthandler, say) runs.
struct sigaction g_prev_segv, g_prev_bus, g_prev_abrt;
void segv_trace(int sig, siginfo_t *si, void *uc)
{
    // async-signal-safe after the warm-up at install: no malloc here
    char msg[256];
    const auto *ctx = static_cast<const ucontext_t *>(uc);
    void *pc = ctx ? reinterpret_cast<void *>(ctx->uc_mcontext.gregs[REG_RIP]) : nullptr;
    Dl_info info{};
    const bool named = pc && dladdr(pc, &info) && info.dli_fname;
    char comm[32] = "?";
    {
        char path[64];
        snprintf(path, sizeof path, "/proc/self/task/%ld/comm", (long)syscall(SYS_gettid));
        const int fd = open(path, O_RDONLY);
        if (fd >= 0) {
            const ssize_t r = read(fd, comm, sizeof comm - 1);
            comm[r > 0 ? r - 1 : 0] = 0;
            close(fd);
        }
    }
    const int l = snprintf(msg, sizeof msg, "mk: signal %d at %p in thread %ld (%s), pc %p = %s+%#lx\n", sig,
                           si ? si->si_addr : nullptr, (long)syscall(SYS_gettid), comm, pc,
                           named ? info.dli_fname : "?",
                           named ? (unsigned long)((char *)pc - (char *)info.dli_fbase) : 0ul);
    if (write(2, msg, (size_t)l) < 0) {
    }
    void *frames[64];
    const int n = backtrace(frames, 64);
    backtrace_symbols_fd(frames, n, 2);
    const struct sigaction &prev = sig == SIGSEGV ? g_prev_segv : sig == SIGBUS ? g_prev_bus : g_prev_abrt;
    if ((prev.sa_flags & SA_SIGINFO) && prev.sa_sigaction) {
        prev.sa_sigaction(sig, si, uc);
        return;
    }
    signal(sig, SIG_DFL);
    raise(sig);
}
struct SegvTrace {
    SegvTrace()
    {
        const char *e = std::getenv("MK_SEGV_TRACE");
        if (!e || *e != '1') return;
        void *warm[2];
        (void)backtrace(warm, 2); // loads the unwinder now, not inside the handler
        struct sigaction sa;
        std::memset(&sa, 0, sizeof sa);
        sa.sa_sigaction = segv_trace;
        sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
        sigaction(SIGSEGV, &sa, &g_prev_segv);
        sigaction(SIGBUS, &sa, &g_prev_bus);
        sigaction(SIGABRT, &sa, &g_prev_abrt);
        on = true;
    }
    bool on = false;
} g_segv_trace;

// Diagnostics: a compiler that installed its own fatal-signal handlers is
// named, and ours put back in front of them.
void segv_trace_check()
{
    if (!g_segv_trace.on) return;
    struct sigaction cur;
    if (sigaction(SIGSEGV, nullptr, &cur) || cur.sa_sigaction == segv_trace) return;
    Dl_info info{};
    const bool named = dladdr(reinterpret_cast<void *>(cur.sa_sigaction), &info) && info.dli_fname;
    fprintf(stderr, "mk: SIGSEGV handler replaced by %s; reinstalled\n", named ? info.dli_fname : "?");
    struct sigaction sa;
    std::memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = segv_trace;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigaction(SIGSEGV, &sa, &g_prev_segv);
    sigaction(SIGBUS, &sa, &g_prev_bus);
    sigaction(SIGABRT, &sa, &g_prev_abrt);
}

// Compile threads: detached, with a stack of their own size.  Clang and LLVM
// recurse deeply on long generated sources; a thread's default stack is the
// stack rlimit (8 MiB here) or 2 MiB where that rlimit is unlimited, less
// than the main thread of a compiler process gets.  With MK_SEGV_TRACE the
// thread also gets an alternate signal stack, so an overflow is reported.
constexpr size_t kCompileStack = (size_t)256 << 20;

void *compile_thread_main(void *arg)
{
    std::unique_ptr<std::function<void()>> f(static_cast<std::function<void()> *>(arg));
    if (g_segv_trace.on) {
        stack_t ss{};
        ss.ss_size = 1 << 16;
        ss.ss_sp = std::malloc(ss.ss_size); // held for the thread's life
        if (ss.ss_sp) (void)sigaltstack(&ss, nullptr);
    }
    (*f)();
    return nullptr;
}

bool spawn_compile_thread(std::function<void()> fn)
{
    auto *f = new std::function<void()>(std::move(fn));
    pthread_attr_t a;
    pthread_attr_init(&a);
    pthread_attr_setstacksize(&a, kCompileStack);
    pthread_attr_setdetachstate(&a, PTHREAD_CREATE_DETACHED);
    pthread_t t;
    const int rc = pthread_create(&t, &a, compile_thread_main, f);
    pthread_attr_destroy(&a);
    if (rc) {
        // no thread: run here (the caller's stack)
        std::unique_ptr<std::function<void()>> own(f);
        (*own)();
        return false;
    }
    return true;
}

std::mutex g_rtc_mu;
std::condition_variable g_rtc_cv;
int g_rtc_running = 0;
void rtc_drain_at_exit()
{
    std::unique_lock<std::mutex> lk(g_rtc_mu);
    (void)g_rtc_cv.wait_for(lk, std::chrono::seconds(120), [] { return g_rtc_running == 0; });
}
struct RtcDrain {
    ~RtcDrain() { rtc_drain_at_exit(); }
} g_rtc_drain;

// The native tier's compiler is this ROCm install's hiprtc, always: a cgo or
// C caller links it, and so does this library.  But in a process that
// imported PyTorch first, PyTorch's bundled libhiprtc / libamd_comgr (the
// same sonames, an older LLVM) are what the linked hiprtc symbols resolve to
// -- a different compiler, whose code differs from network to network (C4
// D=256: 132 VGPRs against 75).  There this ROCm's libhiprtc is opened a
// second time in a link-map namespace of its own (dlmopen LM_ID_NEWLM: its
// libamd_comgr, libstdc++ and libc come with it, invisible to the rest of
// the process), and the module is compiled in process by that copy, so
// every caller gets the same module without a child process.
//
// Round 3 compiled such modules in a child process (posix_spawn from a
// compile thread of a GPU-initialised process); the host heap of those
// PyTorch processes was found corrupted at exit.  Round 5
// removed that path: this library starts no process.  MK_HIPRTC=linked
// compiles with whatever hiprtc the process resolved (PyTorch's in a PyTorch
// process), MK_HIPRTC=ns with the namespace copy; any other value is refused
// (the network stays on tier 2, the plan says why).
#ifndef MK_ROCM_LIB
#define MK_ROCM_LIB "/opt/rocm/lib"
#endif

enum RtcKind { RTC_LINKED, RTC_NS, RTC_REFUSED };

struct RtcChoice {
    RtcKind kind = RTC_LINKED;
    std::string why; // RTC_REFUSED: the reason
};

// Whether the linked hiprtc is another install's than this ROCm's (PyTorch's
// bundled one in a process that imported it first).
bool inproc_rtc_differs()
{
    Dl_info info{};
    if (!dladdr(reinterpret_cast<void *>(&hiprtcCompileProgram), &info) || !info.dli_fname) return false;
    char real[PATH_MAX], want[PATH_MAX];
    if (!realpath(info.dli_fname, real) || !realpath(MK_ROCM_LIB, want)) return true;
    const size_t n = std::strlen(want);
    return std::strncmp(real, want, n) != 0 || real[n] != '/';
}

RtcChoice rtc_choice()
{
    RtcChoice c;
    const char *e = std::getenv("MK_HIPRTC");
    if (e && *e) {
        if (!std::strcmp(e, "linked")) return c;
        if (!std::strcmp(e, "ns")) {
            c.kind = RTC_NS;
            return c;
        }
        c.kind = RTC_REFUSED; // the round-3 helper process (=helper / =<path>) was removed
        c.why = std::string("MK_HIPRTC=") + e + " refused: only linked and ns compile (no helper process)";
        return c;
    }
    if (inproc_rtc_differs()) c.kind = RTC_NS;
    return c;
}

// The hiprtc entry points one compile uses: the linked ones, or this ROCm's
// in its own namespace.
struct RtcApi {
    decltype(&hiprtcCreateProgram) create;
    decltype(&hiprtcCompileProgram) compile;
    decltype(&hiprtcGetProgramLogSize) log_size;
    decltype(&hiprtcGetProgramLog) log;
    decltype(&hiprtcGetCodeSize) code_size;
    decltype(&hiprtcGetCode) code;
    decltype(&hiprtcDestroyProgram) destroy;
    decltype(&hiprtcGetErrorString) error;
    char ***environ_ns = nullptr; // the namespace libc's environ (null: the linked one)
};

const RtcApi kLinkedRtc = {&hiprtcCreateProgram, &hiprtcCompileProgram, &hiprtcGetProgramLogSize,
                           &hiprtcGetProgramLog, &hiprtcGetCodeSize,    &hiprtcGetCode,
                           &hiprtcDestroyProgram, &hiprtcGetErrorString};

void rtc_drain_at_exit();

// This ROCm's hiprtc in a namespace of its own, opened once per process and
// never closed; null (with the reason) when it cannot be opened.
// Namespaces the compiler may open: one per compile worker (NsPool).
constexpr size_t kNsMax = 4;

// This ROCm's libhiprtc: the versioned sonames under MK_ROCM_LIB, highest
// first (libhiprtc.so.7 on ROCm 7.x), then the unversioned link.
std::vector<std::string> hiprtc_candidates()
{
    std::vector<std::string> v;
    glob_t g{};
    if (glob(MK_ROCM_LIB "/libhiprtc.so.[0-9]*", 0, nullptr, &g) == 0)
        for (size_t i = 0; i < g.gl_pathc; i++) v.emplace_back(g.gl_pathv[i]);
    globfree(&g);
    // libhiprtc.so.7 before libhiprtc.so.7.2.x: the soname before the file
    std::sort(v.begin(), v.end(), [](const std::string &a, const std::string &b) {
        return a.size() != b.size() ? a.size() < b.size() : a > b;
    });
    v.emplace_back(MK_ROCM_LIB "/libhiprtc.so");
    return v;
}

// This ROCm's hiprtc in namespace k, opened on first use (by worker k's
// thread, see NsCompiler).
const RtcApi *ns_rtc(size_t k, std::string &why)
{
    static std::string fail[kNsMax];
    static const RtcApi *api[kNsMax];
    static std::once_flag once[kNsMax];
    std::call_once(once[k], [k] { api[k] = [k]() -> const RtcApi * {
        void *h = nullptr;
        std::string errs;
        for (const std::string &path : hiprtc_candidates()) {
            if ((h = dlmopen(LM_ID_NEWLM, path.c_str(), RTLD_NOW | RTLD_LOCAL))) break;
            const char *d = dlerror();
            errs += (errs.empty() ? "" : "; ") + std::string(d ? d : path + ": failed");
        }
        if (!h) {
            fail[k] = "dlmopen: " + errs;
            return nullptr;
        }
        auto *a = new RtcApi{};
        a->create = reinterpret_cast<decltype(a->create)>(dlsym(h, "hiprtcCreateProgram"));
        a->compile = reinterpret_cast<decltype(a->compile)>(dlsym(h, "hiprtcCompileProgram"));
        a->log_size = reinterpret_cast<decltype(a->log_size)>(dlsym(h, "hiprtcGetProgramLogSize"));
        a->log = reinterpret_cast<decltype(a->log)>(dlsym(h, "hiprtcGetProgramLog"));
        a->code_size = reinterpret_cast<decltype(a->code_size)>(dlsym(h, "hiprtcGetCodeSize"));
        a->code = reinterpret_cast<decltype(a->code)>(dlsym(h, "hiprtcGetCode"));
        a->destroy = reinterpret_cast<decltype(a->destroy)>(dlsym(h, "hiprtcDestroyProgram"));
        a->error = reinterpret_cast<decltype(a->error)>(dlsym(h, "hiprtcGetErrorString"));
        a->environ_ns = reinterpret_cast<char ***>(dlsym(h, "__environ"));
        if (!a->create || !a->compile || !a->log_size || !a->log || !a->code_size || !a->code || !a->destroy ||
            !a->error || !a->environ_ns) {
            fail[k] = "dlmopen: hiprtc symbols missing";
            delete a;
            return nullptr;
        }
        // The namespace's static destructors were registered with exit()
        // while it loaded; a compile still running must end before they run,
        // so this drain (registered after them) runs first.
        (void)std::atexit(rtc_drain_at_exit);
        return a;
    }(); });
    why = fail[k];
    return api[k];
}

// Every compile in a namespace runs on one thread, which also opens it, and
// which never exits.  The namespace's libc keeps per-thread state (ctype
// tables, malloc's thread cache, thread_local destructor lists) that only
// the opening thread gets initialised, and that threads started by the
// process's own libc leave behind unrun when they end: compiles on
// short-lived threads crashed now and then in comgr (r04a, CPU reproduction).
class NsCompiler {
  public:
    explicit NsCompiler(size_t k) : k_(k) { spawn_compile_thread([this] { loop(); }); }
    size_t index() const { return k_; }
    // Queues f for the compile thread and returns when it has run.
    void run(const std::shared_ptr<HiprtcJob> &j, const std::function<void()> &f)
    {
        auto done = std::make_shared<std::pair<std::mutex, std::condition_variable>>();
        bool finished = false;
        {
            std::lock_guard<std::mutex> lk(mu_);
            q_.push_back({j, [&f, &finished, done] {
                              f();
                              std::lock_guard<std::mutex> g(done->first);
                              finished = true;
                              done->second.notify_all();
                          }});
        }
        cv_.notify_one();
        std::unique_lock<std::mutex> lk(done->first);
        done->second.wait(lk, [&] { return finished; });
    }
    // Busy with a compile its caller has given up on (rtc_compile's bound):
    // a job queued here would wait for it.
    bool stuck()
    {
        std::shared_ptr<HiprtcJob> cur;
        {
            std::lock_guard<std::mutex> lk(mu_);
            cur = cur_;
        }
        if (!cur) return false;
        std::lock_guard<std::mutex> g(cur->mu);
        return cur->abandoned;
    }

  private:
    void loop()
    {
        for (;;) {
            std::pair<std::shared_ptr<HiprtcJob>, std::function<void()>> job;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [this] { return !q_.empty(); });
                job = std::move(q_.front());
                q_.pop_front();
                cur_ = job.first;
            }
            job.second();
            {
                std::lock_guard<std::mutex> lk(mu_);
                cur_.reset();
            }
            segv_trace_check();
        }
    }
    size_t k_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::pair<std::shared_ptr<HiprtcJob>, std::function<void()>>> q_;
    std::shared_ptr<HiprtcJob> cur_; // the job running now (under mu_)
};

// The namespace compile workers.  A compile that outlives its bound keeps
// its worker (and that copy of LLVM) busy until it ends; the next compile
// goes to the first worker that is not stuck so, opening another namespace
// (up to kNsMax) when all are -- before, one pathological module held up
// every later network's compile until its own bound, each then falling
// back to tier 2 (r05c: a 282-variant census network).  Workers never exit.
class NsPool {
  public:
    static NsPool &get()
    {
        static NsPool *p = new NsPool(); // never destroyed: the threads outlive every caller
        return *p;
    }
    NsCompiler &pick()
    {
        std::lock_guard<std::mutex> lk(mu_);
        for (NsCompiler *w : ws_)
            if (!w->stuck()) return *w;
        if (ws_.size() < kNsMax) {
            ws_.push_back(new NsCompiler(ws_.size()));
            return *ws_.back();
        }
        return *ws_.front(); // all stuck: wait behind the first
    }

  private:
    std::mutex mu_;
    std::vector<NsCompiler *> ws_;
};

// A linked (in-process, this namespace) compile that outlived its bound:
// the next compile takes a namespace worker instead of queueing behind it
// in the same comgr.
std::mutex g_linked_mu;
std::vector<std::weak_ptr<HiprtcJob>> g_linked_running;

bool linked_stuck()
{
    std::lock_guard<std::mutex> lk(g_linked_mu);
    for (auto &w : g_linked_running)
        if (auto j = w.lock()) {
            std::lock_guard<std::mutex> g(j->mu);
            if (j->abandoned && !j->done) return true;
        }
    return false;
}

bool write_file(const std::string &path, const std::string &data)
{
    const int fd = open(path.c_str(), O_WRONLY | O_CREAT | O_EXCL | O_CLOEXEC, 0600);
    if (fd < 0) return false;
    size_t off = 0;
    while (off < data.size()) {
        const ssize_t w = write(fd, data.data() + off, data.size() - off);
        if (w < 0 && errno == EINTR) continue;
        if (w <= 0) break;
        off += (size_t)w;
    }
    return close(fd) == 0 && off == data.size();
}

// Code object version of the native tier's modules: v5, which every HIP runtime a caller may bring understands.  ROCm
// 7.2's hiprtc defaults to v6; loaded into PyTorch's bundled (ROCm 7.0) HIP
// runtime, v6 modules of the machine shape left the host heap corrupted at
// process exit (free(): corrupted unsorted chunks after 60 dynamic-stack
// networks, r03c-r03k), v5 ones and the bundled compiler's did not.
constexpr const char *kCodeObjectVersion = "-mcode-object-version=5";

// The namespace's libc took the process's environment pointer when it was
// opened, and setenv (os.environ[...] = ... in Python) later reallocates and
// frees that array: comgr's getenv then read freed memory (r04: SIGSEGV in
// the compile thread after a test's monkeypatch.setenv).  Each compile gives
// the namespace a private copy of the environment instead: copied from
// `environ` on the caller's thread when the compile is requested
// (rtc_compile, so no compile thread walks the process's array while another
// thread may setenv), installed by the compile thread, which alone reads it.
std::vector<std::string> environ_snapshot()
{
    std::vector<std::string> s;
    for (char **e = environ; e && *e; ++e) s.emplace_back(*e);
    return s;
}

void ns_environ_install(const RtcApi &rt, const std::vector<std::string> &snapshot)
{
    // one copy per namespace (its worker alone refreshes it): a refresh for
    // one namespace must not free the strings another's compile still reads
    struct Env {
        std::vector<std::string> strings;
        std::vector<char *> ptrs;
    };
    static std::mutex mu;
    static std::map<char ***, Env> envs;
    Env *env;
    {
        std::lock_guard<std::mutex> lk(mu);
        env = &envs[rt.environ_ns]; // map nodes are stable
    }
    std::vector<std::string> &strings = env->strings;
    std::vector<char *> &ptrs = env->ptrs;
    std::vector<std::string> s(snapshot);
    std::vector<char *> p;
    p.reserve(s.size() + 1);
    for (std::string &x : s) p.push_back(&x[0]);
    p.push_back(nullptr);
    *rt.environ_ns = p.data(); // the new copy is complete before the old one goes
    strings.swap(s);
    ptrs.swap(p);
}

// In-process hiprtc (the linked symbols, or this ROCm's namespace copy).
void rtc_inproc(const RtcApi &rt, const HiprtcJob &j, bool &ok, std::string &why, std::vector<char> &code)
{
    if (rt.environ_ns) ns_environ_install(rt, j.env);
    const std::string &src = j.src;
    hiprtcProgram prog;
    if (rt.create(&prog, src.c_str(), "mk_jit.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
        why = "hiprtcCreateProgram failed";
        return;
    }
    const char *opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", kCodeObjectVersion};
    const hiprtcResult r = rt.compile(prog, 4, opts);
    size_t cs = 0;
    if (r != HIPRTC_SUCCESS) {
        size_t ls = 0;
        (void)rt.log_size(prog, &ls);
        std::string log(ls, '\0');
        if (ls) (void)rt.log(prog, &log[0]);
        why = std::string("hiprtc: ") + rt.error(r) + ": " + log.substr(0, 400);
    } else if (rt.code_size(prog, &cs) != HIPRTC_SUCCESS || cs == 0) {
        why = "hiprtc produced no code";
    } else {
        code.resize(cs);
        (void)rt.code(prog, code.data());
        ok = true;
    }
    (void)rt.destroy(&prog);
}

bool rtc_abandoned(HiprtcJob &j)
{
    std::lock_guard<std::mutex> lk(j.mu);
    return j.abandoned;
}

// The namespace compiler could not be opened (its reason, e.g. the dlmopen
// error): modules then come from the linked hiprtc ("linked-other" in a
// PyTorch process, whose code differs).  Said once on stderr
// and kept for mk_net_plan (rtc_ns_error=).
std::mutex g_ns_fail_mu;
std::string g_ns_fail;

void ns_degraded(const std::string &why)
{
    std::lock_guard<std::mutex> lk(g_ns_fail_mu);
    if (!g_ns_fail.empty()) return;
    g_ns_fail = why.empty() ? std::string("namespace compiler unavailable") : why;
    fprintf(stderr, "mk: native-tier namespace compiler unavailable (%s); compiling with the linked hiprtc\n",
            g_ns_fail.c_str());
}

std::string ns_fail_reason()
{
    std::lock_guard<std::mutex> lk(g_ns_fail_mu);
    return g_ns_fail;
}

// One compile with the chosen compiler.  The linked hiprtc is the fallback
// when the chosen one cannot run -- unless the caller has given up by then,
// whose result nobody would read.
void hiprtc_run(const std::shared_ptr<HiprtcJob> &j)
{
    bool ok = false;
    std::string why;
    std::vector<char> code;
    const RtcChoice ch = rtc_choice();
    bool ran = false;
    std::string from;
    if (ch.kind == RTC_REFUSED) {
        ran = true; // nothing compiles: the network stays on tier 2
        why = ch.why;
    } else if (ch.kind == RTC_NS || (ch.kind == RTC_LINKED && linked_stuck())) {
        NsCompiler &w = NsPool::get().pick();
        w.run(j, [&] {
            if (const RtcApi *rt = ns_rtc(w.index(), why)) {
                rtc_inproc(*rt, *j, ok, why, code);
                ran = true;
                from = "ns";
            }
        });
        if (!ran) ns_degraded(why);
    }
    if (!ran && !rtc_abandoned(*j)) {
        why.clear();
        {
            std::lock_guard<std::mutex> lk(g_linked_mu);
            g_linked_running.erase(std::remove_if(g_linked_running.begin(), g_linked_running.end(),
                                                  [](const std::weak_ptr<HiprtcJob> &w) { return w.expired(); }),
                                   g_linked_running.end());
            g_linked_running.push_back(j);
        }
        rtc_inproc(kLinkedRtc, *j, ok, why, code);
        from = inproc_rtc_differs() ? "linked-other" : "linked";
    }
    if (ok) why = from; // which compiler's module (mk_net_plan)
    {
        std::lock_guard<std::mutex> lk(j->mu);
        j->ok = ok;
        j->why = std::move(why);
        j->code = std::move(code);
        j->done = true;
        j->cv.notify_all();
    }
    std::lock_guard<std::mutex> lk(g_rtc_mu);
    --g_rtc_running;
    g_rtc_cv.notify_all();
}

uint64_t src_hash(const std::string &src)
{
    uint64_t h = 0xcbf29ce484222325ull; // FNV-1a
    for (unsigned char ch : src) h = (h ^ ch) * 0x100000001b3ull;
    return h;
}

// One module through hiprtc_run on a compile thread, abandoned after max_s
// seconds (`why` says so).  `from` = which compiler built it.
bool rtc_compile(const std::string &src, double max_s, std::vector<char> &code, std::string &why, std::string &from)
{
    auto job = std::make_shared<HiprtcJob>();
    job->src = src;
    job->env = environ_snapshot(); // on the caller's thread (ns_environ_install)
    if (const char *d = std::getenv("MK_JIT_DUMP_SRC"); d && *d) { // diagnostics: every source, before it compiles
        char name[64];
        snprintf(name, sizeof name, "/%016llx.hip", (unsigned long long)src_hash(src));
        (void)write_file(std::string(d) + name, src);
    }
    {
        std::lock_guard<std::mutex> lk(g_rtc_mu);
        ++g_rtc_running;
    }
    spawn_compile_thread([job] { hiprtc_run(job); });
    std::unique_lock<std::mutex> lk(job->mu);
    const auto limit = std::chrono::duration<double>(max_s);
    if (!job->cv.wait_for(lk, limit, [&] { return job->done; })) {
        job->abandoned = true; // the compile runs out in the background, its result discarded
        char b[128];
        snprintf(b, sizeof b, "hiprtc did not finish within the native tier's compile bound (%.0f s)", max_s);
        why = b;
        return false;
    }
    if (!job->ok) {
        why = job->why;
        return false;
    }
    code = std::move(job->code);
    from = job->why; // the compiler whose module this is (hiprtc_run)
    return true;
}

// A numeric field of a code object's AMDGPU metadata (the msgpack note:
// ".vgpr_count", ".agpr_count", ".private_segment_fixed_size"; the native
// modules hold one kernel), or -1.
int64_t co_meta(const std::vector<char> &co, const char *key)
{
    const size_t n = std::strlen(key);
    if (!n || n > 31) return -1;
    const std::string pat = std::string(1, (char)(0xa0u | (unsigned)n)) + key, img(co.begin(), co.end());
    const size_t at = img.find(pat);
    if (at == std::string::npos || at + pat.size() >= img.size()) return -1;
    const size_t i = at + pat.size();
    const uint8_t b = (uint8_t)img[i];
    auto be = [&](size_t k) -> int64_t {
        if (i + k >= img.size()) return -1;
        uint64_t v = 0;
        for (size_t j = 1; j <= k; ++j) v = v << 8 | (uint8_t)img[i + j];
        return (int64_t)v;
    };
    if (b < 0x80u) return b;
    if (b == 0xccu) return be(1);
    if (b == 0xcdu) return be(2);
    if (b == 0xceu) return be(4);
    return -1;
}

// Whether a module holds `waves` waves per SIMD: VGPRs + AGPRs in 8-register
// granules within gfx950's 512 per SIMD lane (`vgpr_file`:
// JitLimits::vgpr_file, lowered only by the tests that take the fallback
// path), and no scratch.  `note` says what was found.
bool module_holds(const std::vector<char> &co, uint32_t waves, uint32_t vgpr_file, std::string &note)
{
    const int64_t v = co_meta(co, ".vgpr_count"), a = co_meta(co, ".agpr_count"),
                  ps = co_meta(co, ".private_segment_fixed_size");
    const int64_t alloc = (v + 7) / 8 * 8 + (std::max<int64_t>(a, 0) + 7) / 8 * 8;
    char b[96];
    snprintf(b, sizeof b, "w%u:v%lld,a%lld,s%lld", waves, (long long)v, (long long)a, (long long)ps);
    note = b;
    return v >= 0 && ps == 0 && alloc * (int64_t)waves <= (int64_t)vgpr_file;
}

// Caller holds h->mu.  Generates and compiles once per SchedCache (hiprtc,
// gfx950); the code object is loaded per device on first use.  Bounded:
// a lane source over lim.max_src_bytes is not compiled, and a compile that
// takes longer than lim.max_compile_s is abandoned -- either way the
// network stays on tier 2 with the reason in mk_net_plan.  A schedule tuned
// for more waves per SIMD (StackPlan::waves) whose module cannot hold them
// (or does not compile) gives way to the next plan (more_waves).
bool jit_compile(SchedCache *sc, const JitLimits &lim)
{
    JitState &J = sc->jit;
    if (J.tried) return J.ok;
    J.tried = true;
    if (!sc->ok) {
        J.why = "no compiled schedule (" + sc->why + ")";
        return false;
    }
    if (lim.disabled) {
        J.why = "disabled by MK_JIT=0";
        return false;
    }
    const auto t0 = std::chrono::steady_clock::now();
    int compiles = 0;
    for (;;) {
        JitLimits L = lim; // the network's LDS budget, when the loader chose one (tune_lds_auto)
        if (sc->lds_set) L.lds_slot_bytes = sc->lds_bytes;
        if (sc->max_dops) L.max_dops = std::max(L.max_dops, sc->max_dops);
        std::string lane, note;
        bool ok = jit_lane_source(sc->prog, L, lane, J.why, &J.shape, &J.max_steps, &J.heavy, false, &J.pool);
        std::string src;
        if (ok) {
            // machine modules: the tile the launch sizes its grid by (MK_TS_R)
            if (J.shape == JIT_MACHINE) L.ts_rounds = jit_sort_rounds(L, sc->prog.nslots);
            J.heavy = J.heavy && J.shape == JIT_STREAM;
            J.lds = jit_slots_in_lds(sc->prog.nslots, J.heavy, L);
            J.lds_n = J.heavy ? jit_lds_slot_count(sc->prog.nslots, J.heavy, L) : 0u;
            J.block = J.heavy ? kJitHeavyBlock : J.pool >= 64 ? kJitPoolBlock : kJitBlock;
            src = jit_module_source(lane, J.shape, J.heavy, L, J.pool);
            J.src_bytes = src.size();
            J.src_hash = src_hash(src);
            // one wall-clock bound for all the plans' compiles together (the
            // first compile gets at least a tenth of it; a later plan none
            // when it is spent, and the network stays on tier 2)
            const double left = lim.max_compile_s -
                                std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (compiles && left <= 0.0) {
                ok = false;
                J.why += "; no time left for the next stack plan";
                sc->alts.clear();
            } else {
                ok = rtc_compile(src, std::max(left, 0.1 * lim.max_compile_s), J.code, J.why, J.rtc);
                ++compiles;
            }
        }
        if (sc->want_waves) {
            const bool held = ok && module_holds(J.code, sc->want_waves, lim.vgpr_file, note);
            sc->occ_note += (sc->occ_note.empty() ? "" : ";") + (ok ? note : "w" + std::to_string(sc->want_waves) + ":declined") +
                            (held ? "" : "-rejected");
            if (!held && !sc->alts.empty()) { // the next plan
                StackPlan next = std::move(sc->alts.front());
                sc->alts.erase(sc->alts.begin());
                use_plan(sc, std::move(next));
                sc->tile = sched_default_tile(sc->prog);
                J.code.clear(); // (tier 2 kept the default plan throughout: tier2_prog)
                continue;
            }
        }
        if (!ok) return false;
        if (const char *d = std::getenv("MK_JIT_DUMP"); d && *d) { // diagnostics: the code object, as loaded,
            if (FILE *f = std::fopen(d, "wb")) {                   // and its source beside it (<path>.hip)
                std::fwrite(J.code.data(), 1, J.code.size(), f);
                std::fclose(f);
            }
            if (FILE *f = std::fopen((std::string(d) + ".hip").c_str(), "wb")) {
                std::fwrite(src.data(), 1, src.size(), f);
                std::fclose(f);
            }
        }
        break;
    }
    sc->alts.clear(); // the plan is settled
    J.compile_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    J.ok = true;
    return true;
}

// Caller holds h->mu.
int ensure_jit_device(SchedCache *sc, int d)
{
    JitDev &jd = sc->jit.dev[d];
    if (jd.fn) return MK_OK;
    DeviceGuard g(d);
    if (load_module(d, sc->jit.code, sc->jit.rtc, &jd.mod) != hipSuccess) return MK_EDEVICE;
    if (hipModuleGetFunction(&jd.fn, jd.mod, kJitKernel) != hipSuccess) return MK_EDEVICE;
    if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&jd.per_cu, jd.fn, sc->jit.block, 0) != hipSuccess ||
        jd.per_cu < 1)
        jd.per_cu = 1;
    // The occupancy API ignores part of the SGPR cost on ROCm 7.2: resident
    // waves per SIMD are at most 800 / (ceil(sgpr / 16) * 16 + 16)
    // (MI355X_MICROARCH.md; 82-96 SGPRs admit 7 where the API says 8).  A
    // grid sized by the API's answer leaves a tail of blocks that run only
    // after others finish.
    if (const int64_t sg = co_meta(sc->jit.code, ".sgpr_count"); sg > 0) {
        const int per_simd = 800 / ((int)((sg + 15) / 16) * 16 + 16);
        const int cap = std::max(1, per_simd * 4 / std::max(1, sc->jit.block / 64));
        jd.per_cu = std::min(jd.per_cu, cap);
    }
    if (const char *e = std::getenv("MK_JIT_PER_CU"); e && *e) // diagnostics: blocks per CU of the grid
        jd.per_cu = std::max(1, std::atoi(e));

    if (std::getenv("MK_JIT_SHOW_GRID"))
        fprintf(stderr, "mk: native kernel on device %d: %d blocks of %d per CU\n", d, jd.per_cu, sc->jit.block);
    return MK_OK;
}

// Host-API calls of up to this many inputs per device stage through pinned
// memory (4M); MK_HOST_CHUNK overrides it for networks loaded afterwards.
uint64_t host_chunk_from_env()
{
    const char *e = std::getenv("MK_HOST_CHUNK");
    const unsigned long long x = e ? std::strtoull(e, nullptr, 10) : 0ull;
    return x ? (uint64_t)x : (uint64_t)1 << 22;
}

// GridTune: batches from this size on are tuned (smaller ones run the
// resident grid; their launches are short and their grid often not full)
constexpr uint64_t kGridTuneMin = uint64_t(1) << 18;

struct GridPick {
    int blocks = 0;
    int timed = -1; // candidate whose events bracket this launch, or -1
};

// One launch's grid under GridTune (`resident`: the untuned grid).
GridPick grid_tune_pick(GridTune &t, uint64_t n, int resident)
{
    GridPick g;
    g.blocks = resident;
    if (t.n != n || t.cand[2] != resident) {
        t.n = n;
        t.phase = 0;
        t.cand[0] = std::max(1, resident * 3 / 4);
        t.cand[1] = std::max(1, resident / 2);
        t.cand[2] = resident;
        t.chosen = resident;
    }
    if (t.phase < 3) {
        for (hipEvent_t &e : t.ev)
            if (!e && hipEventCreate(&e) != hipSuccess) {
                t.phase = 4; // no events: the resident grid
                return g;
            }
        g.timed = t.phase;
        g.blocks = t.cand[t.phase++];
        return g;
    }
    if (t.phase == 3) {
        if (hipEventQuery(t.ev[5]) != hipSuccess) return g; // not measured yet: never wait
        bool ok = true;
        for (int k = 0; k < 3; k++) ok = ok && hipEventElapsedTime(&t.ms[k], t.ev[2 * k], t.ev[2 * k + 1]) == hipSuccess;
        // a smaller grid is kept only when it is clearly faster (5%)
        int best = 2;
        for (int k = 0; k < 2; k++)
            if (ok && t.ms[k] > 0.f && t.ms[k] < 0.95f * t.ms[2] && t.ms[k] < t.ms[best]) best = k;
        t.chosen = t.cand[best];
        t.phase = 4;
    }
    g.blocks = t.chosen;
    return g;
}

// Caller holds h->mu.  Tier-3 launch; asynchronous on `stream`.
int launch_jit_locked(mk_net *h, SchedCache *sc, int d, const mk_input *in, size_t n, int32_t *d_out,
                      uint8_t *d_status, uint32_t *d_steps, uint64_t *d_stats, uint32_t budget, uint32_t flags,
                      hipStream_t stream)
{
    int rc = ensure_jit_device(sc, d);
    if (rc) return rc;
    DevCtx &c = h->dev[d];
    SchedDev &sd = sc->dev[d];
    JitDev &jd = sc->jit.dev[d];
    const SchedProgram &P = sc->prog;
    DeviceGuard g(d);
    const uint64_t block = (uint64_t)sc->jit.block;
    const bool heavy = sc->jit.shape == JIT_STREAM && sc->jit.heavy;
    // stack slots in HBM (none when the heavy kernel keeps them in LDS)
    const uint32_t nslots = P.nslots - sc->jit.lds_n;
    // heavy: one thread per input, `chunk` inputs per launch (slot memory);
    // otherwise a resident grid whose threads loop over the inputs
    uint64_t chunk = n, lanes;
    int blocks, alloc_blocks = 0;
    GridPick tune;
    if (heavy) {
        if (nslots) {
            const uint64_t fit = h->jit_lim.slot_bytes / ((uint64_t)nslots * sizeof(int32_t));
            chunk = std::min<uint64_t>(n, std::max<uint64_t>(block, fit / block * block));
        }
        lanes = (std::max<uint64_t>(chunk, 1) + block - 1) / block * block;
        blocks = (int)(lanes / block);
    } else {
        // inputs a block takes: the stream kernel's tile, the tile-sorted
        // machine kernel's (a block holds at least one full tile), else one
        // per thread
        const bool sorted = sc->jit.shape == JIT_MACHINE && !sc->jit.pool && h->jit_lim.tile_sort && !h->jit_lim.order;
        const uint64_t per_block = sc->jit.shape == JIT_STREAM ? block * kJitStreamLanes
                                   : sorted ? block * jit_sort_rounds(h->jit_lim, P.nslots)
                                            : block;
        const uint64_t want = (n + per_block - 1) / per_block;
        const uint64_t resident = (uint64_t)jd.per_cu * (uint64_t)std::max(c.cus, 1);
        blocks = (int)std::max<uint64_t>(1, std::min<uint64_t>(want, resident));
        if (sc->jit.shape == JIT_MACHINE && nslots) {
            // machine modules address a slot as slot x stride in 24-bit x 24-bit
            // -> 32-bit arithmetic (module_prelude narrow_slots): stride
            // (slot columns) < 2^24 and slots x stride < 2^32
            const uint64_t per = sc->jit.pool >= 64 ? (uint64_t)sc->jit.pool  // slot columns per block (slot_cols below)
                                 : sc->jit.pool ? block * sc->jit.pool : block;
            const uint64_t cap = std::min<uint64_t>(((1ull << 32) - 1) / ((uint64_t)nslots * per), ((1ull << 24) - 1) / per);
            if (cap < 1) return MK_ELIMIT;
            blocks = (int)std::min<uint64_t>((uint64_t)blocks, cap);
        }
        alloc_blocks = blocks;
        if (sorted && nslots && !sc->jit.pool && h->jit_lim.tune_grid && n >= kGridTuneMin) {
            hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
            if (hipStreamIsCapturing(stream, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone) {
                int e = 0;
                while (e < 4 && jd.tune[e].n != n) e++;
                if (e == 4) {
                    e = jd.tune_next;
                    jd.tune_next = (jd.tune_next + 1) % 4;
                }
                jd.tune_last = e;
                tune = grid_tune_pick(jd.tune[e], n, blocks);
                blocks = tune.blocks;
            }
        }
        lanes = (uint64_t)blocks * block;
    }
    // stack-slot columns: one per thread, or (pool kernel) one per pool slot
    const uint64_t slot_cols = sc->jit.pool >= 64 ? (uint64_t)blocks * sc->jit.pool
                               : sc->jit.pool      ? lanes * sc->jit.pool
                                                   : lanes;
    if (nslots) {
        // (sized for the resident grid, so that a tuning launch's smaller
        // grid does not reallocate)
        const size_t need = (size_t)nslots * std::max<uint64_t>(slot_cols, (uint64_t)alloc_blocks * block) * sizeof(int32_t);
        if (need > sd.slots_bytes) {
            if (sd.d_slots) {
                (void)hipDeviceSynchronize();
                (void)hipFree(sd.d_slots);
                sd.d_slots = nullptr;
                sd.slots_bytes = 0;
            }
            if (hipMalloc(&sd.d_slots, need) != hipSuccess) return MK_ENOMEM;
            sd.slots_bytes = need;
        }
    }
    SParams p{};
    p.in_kind = in->kind;
    p.gen_kind = in->gen_kind;
    p.in_data = in->data;
    p.seed = in->seed;
    p.offset = in->offset;
    p.gen_mask = in->gen_mask;
    p.budget = budget;
    p.n = n;
    p.out = d_out;
    p.status = d_status;
    p.steps = d_steps;
    // heavy grids may outnumber the partial rows: their waves add atomically
    if (counting(d_stats, flags) && (rc = ensure_partials(c, heavy ? 0 : lanes))) return rc;
    p.partials = counting(d_stats, flags) ? c.d_partials : nullptr;
    p.part_rows = (uint32_t)(c.partials_bytes / 64);
    p.slots = nslots ? sd.d_slots : nullptr;
    p.lanes = slot_cols;
    p.vlanes = lanes;
    const uintptr_t va = 4u * kJitStreamLanes;
    p.io_vec = in->kind == MK_IN_I32 && (uintptr_t)in->data % va == 0 && (uintptr_t)d_out % va == 0 &&
               (uintptr_t)d_status % kJitStreamLanes == 0 && (uintptr_t)d_steps % va == 0;
    p.order = nullptr;
    if (sc->jit.shape == JIT_MACHINE && !sc->jit.pool && h->jit_lim.order && n >= kOrderMin && n < (1ull << 32)) {
        // group the inputs by value (order_* kernels): lanes of a wave get similar trips
        if (n > sd.order_cap) {
            (void)hipStreamSynchronize(stream);
            (void)hipFree(sd.d_order);
            sd.d_order = nullptr;
            sd.order_cap = 0;
            if (hipMalloc(&sd.d_order, n * sizeof(uint32_t)) != hipSuccess) return MK_ENOMEM;
            sd.order_cap = n;
        }
        if (!sd.d_ordtab && hipMalloc(&sd.d_ordtab, (2 + kOrderBuckets) * sizeof(int32_t)) != hipSuccess)
            return MK_ENOMEM;
        const int32_t init[2] = {INT32_MAX, INT32_MIN};
        const int grid = std::max(1, std::min(c.cus * 8, (int)((n + 255) / 256)));
        if (hipMemsetAsync(sd.d_ordtab + 2, 0, kOrderBuckets * sizeof(int32_t), stream) != hipSuccess ||
            hipMemcpyAsync(sd.d_ordtab, init, sizeof init, hipMemcpyHostToDevice, stream) != hipSuccess)
            return MK_EDEVICE;
        hipLaunchKernelGGL(order_minmax, dim3(grid), dim3(256), 0, stream, p, sd.d_ordtab);
        hipLaunchKernelGGL(order_hist, dim3(grid), dim3(256), 0, stream, p, sd.d_ordtab);
        hipLaunchKernelGGL(order_scan, dim3(1), dim3(1024), 0, stream, sd.d_ordtab);
        hipLaunchKernelGGL(order_scatter, dim3(grid), dim3(256), 0, stream, p, sd.d_ordtab, sd.d_order);
        if (hipGetLastError() != hipSuccess) return MK_EDEVICE;
        p.order = sd.d_order;
    }
    uint64_t s0 = 0;
    do {
        SParams q = p;
        if (heavy) { // inputs s0 .. s0 + q.n - 1
            q.n = std::min<uint64_t>(chunk, n - s0);
            if (in->kind == MK_IN_I64) q.in_data = (const int64_t *)in->data + s0;
            else if (in->kind == MK_IN_I32) q.in_data = (const int32_t *)in->data + s0;
            else q.offset = in->offset + s0;
            q.out = d_out + s0;
            q.status = d_status + s0;
            q.steps = d_steps ? d_steps + s0 : nullptr;
            blocks = (int)std::max<uint64_t>(1, (q.n + block - 1) / block);
        }
        void *args[] = {(void *)&q};
        jd.last_blocks = blocks;
        if (tune.timed >= 0 && hipEventRecord(jd.tune[jd.tune_last].ev[2 * tune.timed], stream) != hipSuccess)
            return MK_EDEVICE;
        if (hipModuleLaunchKernel(jd.fn, blocks, 1, 1, (unsigned)block, 1, 1, 0, stream, args, nullptr) !=
            hipSuccess)
            return MK_EDEVICE;
        if (tune.timed >= 0 && hipEventRecord(jd.tune[jd.tune_last].ev[2 * tune.timed + 1], stream) != hipSuccess)
            return MK_EDEVICE;
    } while (heavy && chunk && (s0 += chunk) < n);
    return fold_now(d_stats, flags) ? launch_stats_reduce(c, d_stats, stream) : MK_OK;
}

enum Tier { TIER_NONE, TIER_INTERP, TIER_COMPILED, TIER_NATIVE };
constexpr uint32_t kSchedInterpSb = 1024; // above: tier 1 instead of tier 2 (pick_tier)

// Caller holds h->mu.  The tier a launch with `flags` runs on: tier 1 when
// forced; else the native kernel unless tier 2 was asked for (TILE/REFILL);
// else the superblock interpreter; tier 1 when the schedule compiler gave up.
// The stream-shaped native kernel has no budget checks: it serves launches
// whose budget exceeds every path of the network; smaller budgets go to tier 2.
Tier pick_tier(mk_net *h, uint32_t cap, uint32_t flags, uint32_t budget, SchedCache **out)
{
    *out = nullptr;
    if (flags & MK_FLAG_FORCE_INTERP) return TIER_INTERP;
    SchedCache *sc = get_sched(h, cap, (flags & MK_FLAG_STOP_ON_OUTPUT) != 0);
    *out = sc;
    const bool want_jit = (flags & MK_FLAG_JIT) || !(flags & (MK_FLAG_TILE | MK_FLAG_REFILL));
    if (want_jit && jit_compile(sc, h->jit_lim) && (sc->jit.shape == JIT_MACHINE || (uint64_t)budget > sc->jit.max_steps))
        return TIER_NATIVE;
    if (flags & MK_FLAG_JIT) return TIER_NONE;
    // A schedule with thousands of superblocks is control state that follows
    // the data (a stack depth per state): tier 2 would dispatch nearly one
    // superblock per lane, and the interpreter is faster (census class
    // data_dependent_stack_depth, 4,098 superblocks: 0.016 T node-instr/s on
    // tier 2, 0.080 T on tier 1).  TILE / REFILL still demand tier 2.
    if (sc->ok && tier2_prog(sc).nsb > kSchedInterpSb && !(flags & (MK_FLAG_TILE | MK_FLAG_REFILL))) return TIER_INTERP;
    return sc->ok ? TIER_COMPILED : TIER_INTERP;
}

// Caller holds h->mu.  Asynchronous on `stream`.
int launch_locked(mk_net *h, int d, const mk_input *in, size_t n, int32_t *d_out, uint8_t *d_status,
                  uint32_t *d_steps, uint64_t *d_stats, const mk_opts *o, hipStream_t stream,
                  mk_trace_entry *trace = nullptr, uint32_t trace_max = 0, uint32_t *trace_n = nullptr)
{
    if (n == 0) return MK_OK;
    int rc = ensure_device(h, d);
    if (rc) return rc;
    DevCtx &c = h->dev[d];
    DeviceGuard g(d);
    if ((rc = order_on(c, stream))) return rc;
    uint32_t budget, cap, flags;
    resolve_opts(o, budget, cap, flags);
    SchedCache *sc = nullptr;
    switch (pick_tier(h, cap, flags, budget, &sc)) {
    case TIER_NATIVE:
        return launch_jit_locked(h, sc, d, in, n, d_out, d_status, d_steps, d_stats, budget, flags, stream);
    case TIER_COMPILED:
        return launch_sched_locked(h, sc, d, in, n, d_out, d_status, d_steps, d_stats, budget, flags, stream);
    case TIER_NONE: return MK_ELIMIT; // native tier demanded but unavailable (mk_net_plan says why)
    default: break;
    }
    Launch L;
    if ((rc = plan_launch(h->net, c, n, cap, L))) return rc;
    const uint64_t lanes = (uint64_t)L.blocks * kBlock;
    uint32_t spill_rows = 0;
    if (h->net.uses_stacks && cap > L.ring) {
        spill_rows = cap - L.ring;
        const size_t need = (size_t)h->net.nstack * spill_rows * lanes * sizeof(int32_t);
        if (need > c.spill_bytes) {
            if (c.d_spill) {
                (void)hipDeviceSynchronize();
                (void)hipFree(c.d_spill);
                c.d_spill = nullptr;
                c.spill_bytes = 0;
            }
            if (hipMalloc(&c.d_spill, need) != hipSuccess) return MK_ENOMEM;
            c.spill_bytes = need;
        }
    }
    KParams p{};
    for (int i = 0; i < h->net.nprog; i++) {
        p.base[i] = h->net.base[i];
        p.len[i] = h->net.len[i];
    }
    p.nprog = h->net.nprog;
    p.nstack = h->net.uses_stacks ? h->net.nstack : 0;
    p.in_kind = in->kind;
    p.in_data = in->data;
    p.seed = in->seed;
    p.gen_kind = in->gen_kind;
    p.gen_mask = in->gen_mask;
    p.offset = in->offset;
    p.n = n;
    p.out = d_out;
    p.status = d_status;
    p.steps = d_steps;
    if (counting(d_stats, flags) && (rc = ensure_partials(c, lanes))) return rc;
    p.partials = counting(d_stats, flags) ? c.d_partials : nullptr;
    p.budget = budget;
    p.stack_cap = cap;
    p.flags = flags;
    p.ring = L.ring;
    p.spill_rows = spill_rows;
    p.spill = c.d_spill;
    p.lanes = lanes;
    p.trace = trace;
    p.trace_max = trace_max;
    p.trace_n = trace_n;
    const Insn *code = c.d_code;
    void *args[] = {(void *)&code, (void *)&p};
    if (hipLaunchKernel(L.fn, dim3(L.blocks), dim3(kBlock), args, L.lds, stream) != hipSuccess)
        return MK_EDEVICE;
    return fold_now(d_stats, flags) ? launch_stats_reduce(c, d_stats, stream) : MK_OK;
}

// ---- stateful sessions: host side -----------------------------------------
template <int NMAX>
void *session_kernel_ptr() { return reinterpret_cast<void *>(&tis_session<NMAX>); }

void *pick_session_kernel(int nprog)
{
    if (nprog <= 1) return session_kernel_ptr<1>();
    if (nprog <= 2) return session_kernel_ptr<2>();
    if (nprog <= 4) return session_kernel_ptr<4>();
    if (nprog <= 8) return session_kernel_ptr<8>();
    return session_kernel_ptr<16>();
}

} // namespace
} // namespace mk

struct mk_session {
    mk_net *h = nullptr;
    int device = 0;
    size_t n = 0;
    uint32_t budget = 0, cap = 0;
    int nprog = 0, nstack = 0;
    std::mutex mu;
    void *d_state = nullptr; // every per-session array, one allocation
    size_t state_bytes = 0;
    void *d_stage = nullptr; // host-API staging: in, out, status, steps
    void *h_stage = nullptr; // pinned host mirror of d_stage
    size_t stage_bytes = 0;
    hipStream_t stream = nullptr;
    mk::SessParams p{};
    // native tier (tis_jit.h mk_sess_exec): the session schedule compiled to
    // a kernel; the interpreter's state above holds the sessions handed to it
    bool native = false;
    // longest call on the native tier (jit_session_max_call_steps): with a
    // budget above it no call hands off, and the interpreter is not launched
    uint64_t call_steps = UINT64_MAX;
    std::string plan; // mk_session_plan
    hipModule_t mod = nullptr;
    hipFunction_t fn = nullptr;
    std::vector<char> code; // the module's code object: HIP may read the image after hipModuleLoadData
    std::string rtc_from;   // its compiler (load_module / release_module)
    void *d_native = nullptr; // every native array, one allocation
    size_t native_bytes = 0;
    uint32_t *nsb = nullptr, *hand_sb = nullptr, *hand_steps = nullptr, *hand_call = nullptr;
    uint32_t *sflags = nullptr; // SessParams::sflags
    uint32_t epoch = 0;         // native launches so far (never 0 after the first)
    // A launch whose native kernel ran but whose import / interpreter launch
    // failed leaves handed-off sessions that no kernel will serve again:
    // every call then fails (MK_EDEVICE) until mk_session_reset.
    bool broken = false;
    hipEvent_t order = nullptr; // recorded after each launch on a caller stream (session_order)
    hipStream_t last = nullptr; // the stream `order` was last recorded on
    int64_t *regs = nullptr;
    int32_t *slots = nullptr;
    mk::SessMapHdr *hdr = nullptr;
    mk::SessSrcDev *rec = nullptr;
    int64_t *dyn_base = nullptr;
    ~mk_session()
    {
        mk::DeviceGuard g(device);
        if (last && order) (void)hipEventSynchronize(order); // the last launch on a caller stream
        if (stream) (void)hipStreamSynchronize(stream);
        (void)hipFree(d_state);
        (void)hipFree(d_native);
        (void)hipFree(d_stage);
        (void)hipHostFree(h_stage);
        mk::release_module(mod, rtc_from);
        if (order) (void)hipEventDestroy(order);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

namespace mk {
namespace {

// Parameters of the native session kernel (tis_jit.cpp kSessionKernel's SessK).
struct SessK {
    uint64_t n;
    uint32_t ncalls, budget;
    const int64_t *in;
    int32_t *out;
    uint8_t *status;
    uint32_t *steps;
    uint32_t *sb;
    int64_t *regs;
    int32_t *slots;
    uint32_t *hand_sb, *hand_steps, *hand_call;
    uint32_t *sflags;
    uint32_t epoch;
};

// *queued (when given) is set once a kernel has been queued on `stream`, so
// that a caller whose launch fails part way still orders later work after it.
// `done` (when given) is recorded by the launch's last kernel itself, as its
// completion event (hipExtModuleLaunchKernel / hipExtLaunchKernel stop
// event), instead of by a separate hipEventRecord after it: that marker cost
// ~3 us of stream time per call (round 6, profiles/r08_sessions_ab.txt).
int session_launch(mk_session *s, const int64_t *d_in, int32_t *d_out, uint8_t *d_status, uint32_t *d_steps,
                   hipStream_t stream, uint32_t ncalls = 1, bool resume = false, bool *queued = nullptr,
                   hipEvent_t done = nullptr)
{
    if (s->broken) return MK_EDEVICE;
    if (s->n == 0 || ncalls == 0) return MK_OK;
    SessParams p = s->p;
    p.ncalls = ncalls;
    p.resume = resume ? 1u : 0u;
    p.in = d_in;
    p.out = d_out;
    p.status = d_status;
    p.steps = d_steps;
    const Insn *code = s->h->dev[s->device].d_code;
    const size_t lds = (size_t)(s->nprog * 4 + s->nstack) * kBlock * 4;
    const uint64_t blocks = (s->n + kBlock - 1) / kBlock;
    if (blocks > 0x7fffffffull) return MK_ELIMIT;
    const uint64_t iblocks = blocks < kSessGridCap ? blocks : kSessGridCap; // the interpreter's grid-stride grid
    if (s->native && !resume) {
        if (++s->epoch == 0) s->epoch = 1; // sflags[0] starts at 0: "no hand-off yet"
        // 1. the native kernel: every session it holds, every call of the burst
        SessK k{s->n, ncalls, p.budget, d_in, d_out, d_status, d_steps, s->nsb, s->regs, s->slots,
                s->hand_sb, s->hand_steps, s->hand_call, s->sflags, s->epoch};
        void *kargs[] = {(void *)&k};
        // the native kernel is the launch's last when the interpreter pass is
        // skipped (below: no call can reach the budget)
        const bool last = s->call_steps < (uint64_t)p.budget;
        if (hipExtModuleLaunchKernel(s->fn, (uint32_t)(blocks * kBlock), 1, 1, kBlock, 1, 1, 0, stream, kargs, nullptr,
                                     nullptr, last ? done : nullptr, 0) != hipSuccess)
            return MK_EDEVICE;
        if (queued) *queued = true;
        // 2. calls it handed off become interpreter sessions: imported by
        // the interpreter kernel itself, thread by thread, before it runs
        p.fuse_import = 1u;
        p.imp = SessImport{s->n, s->nprog, s->nstack, s->nsb, s->sflags, s->epoch, s->hand_sb, s->hand_steps,
                           s->regs, s->slots, s->hdr, s->rec, s->dyn_base};
        // no call of this network can reach the budget: none hands off and
        // the interpreter holds no session, so its pass would only exit
        if (s->call_steps < (uint64_t)p.budget) return MK_OK;
    }
    // 3. the interpreter: its sessions (all of them without the native tier)
    void *args[] = {(void *)&code, (void *)&p};
    if (hipExtLaunchKernel(pick_session_kernel(s->nprog), dim3((unsigned)iblocks), dim3(kBlock), args, lds, stream,
                           nullptr, done, 0) != hipSuccess) {
        if (s->native && !resume) s->broken = true;
        return MK_EDEVICE;
    }
    return MK_OK;
}

// The native tier for a session set (row f2): the session schedule
// (compile_session_schedule), its kernel (jit_session_source + hiprtc), the
// state maps of its superblocks and the per-session lane state.  A network
// the compiler or the native tier declines keeps the interpreter, with the
// reason in s->plan; so does MK_SESSION_NATIVE=0.  Allocation failures are
// errors.
int session_native(mk_session *s)
{
    mk_net *h = s->h;
    auto decline = [&](const std::string &why) {
        s->plan = "tier=interp reason=" + why;
        return MK_OK;
    };
    if (const char *e = std::getenv("MK_SESSION_NATIVE"); e && !std::strcmp(e, "0"))
        return decline("disabled by MK_SESSION_NATIVE=0");
    if (h->jit_lim.disabled) return decline("disabled by MK_JIT=0");
    SchedProgram P;
    std::string why, src, from;
    {
        std::lock_guard<std::mutex> lk(h->mu);
        if (!compile_session_schedule(h->net, s->cap, SchedLimits{}, P, why)) return decline(why);
        if (!jit_session_source(P, h->jit_lim, src, why)) return decline(why);
    }
    if (src.size() > h->jit_lim.max_src_bytes) return decline("session source over the native tier's size bound");
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<char> &code = s->code; // kept while the module is loaded
    if (!rtc_compile(src, h->jit_lim.max_compile_s, code, why, from)) return decline(why);
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    DeviceGuard g(s->device);
    s->rtc_from = from;
    if (load_module(s->device, code, from, &s->mod) != hipSuccess ||
        hipModuleGetFunction(&s->fn, s->mod, kJitSessKernel) != hipSuccess)
        return MK_EDEVICE;
    std::vector<SessMapHdr> hdr;
    std::vector<SessSrcDev> rec;
    build_sess_map(P, s->nprog, s->nstack, hdr, rec);
    const size_t N = s->n ? s->n : 1;
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t sz[] = {al(N * 4), al((size_t)P.nregs * N * 8), al((size_t)std::max<uint32_t>(P.nslots, 1) * N * 4),
                         al(N * 4), al(N * 4), al(N * 4), al(16), al(hdr.size() * sizeof(SessMapHdr)),
                         al(rec.size() * sizeof(SessSrcDev)), al(std::max<size_t>(P.dyn_base.size(), 1) * 8)};
    size_t total = 0;
    for (size_t b : sz) total += b;
    if (hipMalloc(&s->d_native, total) != hipSuccess) return MK_ENOMEM;
    s->native_bytes = total;
    char *b = (char *)s->d_native;
    size_t off = 0;
    auto take = [&](size_t i) { char *q = b + off; off += sz[i]; return q; };
    s->nsb = (uint32_t *)take(0);
    s->regs = (int64_t *)take(1);
    s->slots = (int32_t *)take(2);
    s->hand_sb = (uint32_t *)take(3);
    s->hand_steps = (uint32_t *)take(4);
    s->hand_call = (uint32_t *)take(5);
    s->sflags = (uint32_t *)take(6);
    s->hdr = (SessMapHdr *)take(7);
    s->rec = (SessSrcDev *)take(8);
    s->dyn_base = (int64_t *)take(9);
    // the maps never change: copied once (reset clears only the lane state)
    if ((!hdr.empty() && hipMemcpy(s->hdr, hdr.data(), hdr.size() * sizeof(SessMapHdr), hipMemcpyHostToDevice) !=
                             hipSuccess) ||
        (!rec.empty() && hipMemcpy(s->rec, rec.data(), rec.size() * sizeof(SessSrcDev), hipMemcpyHostToDevice) !=
                             hipSuccess) ||
        (!P.dyn_base.empty() &&
         hipMemcpy(s->dyn_base, P.dyn_base.data(), P.dyn_base.size() * 8, hipMemcpyHostToDevice) != hipSuccess))
        return MK_EDEVICE;
    s->native_bytes = sz[0] + sz[1] + sz[2] + sz[3] + sz[4] + sz[5] + sz[6]; // the lane state: what a reset clears
    s->native = true;
    s->call_steps = jit_session_max_call_steps(P, h->jit_lim);
    s->p.nsb = s->nsb;
    s->p.hand_call = s->hand_call;
    s->p.sflags = s->sflags;
    // registers a launch loads and stores per instance (mk_sess_load's lines):
    // with sb, the state bytes of the sessions' byte model (tools/sess_roofline.py)
    size_t live_regs = 0;
    for (size_t at = src.find("on ? regs["); at != std::string::npos; at = src.find("on ? regs[", at + 1)) ++live_regs;
    char line[320];
    snprintf(line, sizeof line, "tier=native superblocks=%u regs=%u slots=%u words=%zu source=%zuB kernel=%016llx "
             "compile=%.2fs rtc=%s state_regs=%zu", P.nsb, P.nregs, P.nslots, P.code.size(), src.size(),
             (unsigned long long)src_hash(src), secs, from.c_str(), live_regs);
    s->plan = line;
    // calls that cannot reach the budget: one launch per call (no interpreter pass)
    s->plan += s->call_steps < (uint64_t)s->p.budget ? " call_steps=" + std::to_string(s->call_steps) + " launches=1"
                                                     : std::string(" launches=2");
    return MK_OK;
}

void set_err(char *err, size_t len, const std::string &s)
{
    if (!err || !len) return;
    size_t k = std::min(len - 1, s.size());
    memcpy(err, s.data(), k);
    err[k] = 0;
}

int copy_out(char *out, size_t len, const std::string &s)
{
    if (!out || !len) return MK_EINVAL;
    set_err(out, len, s);
    return s.size() < len ? MK_OK : MK_EINVAL;
}

} // namespace
} // namespace mk

// ------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------
extern "C" {

const char *mk_version(void) { return "misaka-net-amd 0.1.0 (gfx950)"; }

int mk_net_load(const mk_node_desc *nodes, int n, mk_net **out, char *err, size_t err_len)
{
    if (!nodes || n <= 0 || !out) {
        mk::set_err(err, err_len, "invalid arguments");
        return MK_EINVAL;
    }
    *out = nullptr;
    std::vector<mk::NodeSpec> specs;
    for (int i = 0; i < n; i++) {
        if (!nodes[i].name) {
            mk::set_err(err, err_len, "node without a name");
            return MK_EINVAL;
        }
        specs.push_back({nodes[i].name, nodes[i].kind, nodes[i].program ? nodes[i].program : ""});
    }
    mk_net *h = new (std::nothrow) mk_net();
    if (!h) return MK_ENOMEM;
    std::string e;
    int rc = mk::lower_network(specs, h->net, e);
    if (rc) {
        mk::set_err(err, err_len, e);
        delete h;
        return rc;
    }
    h->host_chunk = mk::host_chunk_from_env();
    mk::set_err(err, err_len, "");
    *out = h;
    return MK_OK;
}

void mk_net_free(mk_net *net) { delete net; }

int mk_compute_batch(mk_net *h, const int64_t *in, size_t n, int32_t *out, uint8_t *status, uint32_t *steps,
                     const mk_opts *opts)
{
    if (!h || (n && (!in || !out || !status))) return MK_EINVAL;
    if (n == 0) return MK_OK;
    std::lock_guard<std::mutex> lk(h->mu);
    const int ndev = mk::device_count();
    if (ndev <= 0) return MK_EDEVICE;
    // device_mask: the GPUs this process shards the batch over (contiguous
    // ranges); a bit naming a GPU that does not exist is an error
    std::vector<int> devs;
    const uint32_t mask = opts ? opts->device_mask : 0u;
    if (mask == 0) devs.push_back(0);
    for (int d = 0; d < 32; d++)
        if (mask & (1u << d)) {
            if (d >= ndev || d >= mk::kMaxDevices) return MK_EINVAL;
            devs.push_back(d);
        }
    const size_t G = devs.size();
    struct Job { int d; size_t lo, hi; };
    std::vector<Job> jobs;
    for (size_t g = 0; g < G; g++) {
        const size_t lo = n * g / G, hi = n * (g + 1) / G;
        if (hi > lo) jobs.push_back({devs[g], lo, hi});
    }
    // Transfers: a device's share up to one chunk (h->host_chunk inputs, the
    // master's bursts and other latency-bound calls) goes through pinned
    // staging, so each copy is one DMA with no runtime staging or extra sync;
    // larger shares go straight from the caller's pageable buffers, where the
    // runtime's own pipelined staging moves more bytes per second than one
    // host thread copying into pinned memory (C2, 16M lanes: 9.7 ms per call
    // pageable vs 13.2 ms through a single-threaded pinned double buffer).
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    for (auto &j : jobs) {
        int rc = mk::ensure_device(h, j.d);
        if (rc) return rc;
        mk::DevCtx &c = h->dev[j.d];
        mk::DeviceGuard g(j.d);
        const size_t m = j.hi - j.lo;
        const bool pinned = m <= h->host_chunk;
        const size_t a8 = al(m * 8), a4 = al(m * 4), a1 = al(m);
        const size_t need = a8 + a4 + a4 + a1; // in, out, steps, status
        if (need > c.stage_bytes || (pinned && !c.h_stage)) {
            (void)hipStreamSynchronize(c.stream);
            (void)hipFree(c.d_stage);
            (void)hipHostFree(c.h_stage);
            c.d_stage = c.h_stage = nullptr;
            c.stage_bytes = 0;
            const size_t sz = std::max(need, c.stage_bytes);
            if (hipMalloc(&c.d_stage, sz) != hipSuccess) return MK_ENOMEM;
            if (sz <= al(h->host_chunk * 8) + 2 * al(h->host_chunk * 4) + al(h->host_chunk) &&
                hipHostMalloc(&c.h_stage, sz, hipHostMallocDefault) != hipSuccess)
                return MK_ENOMEM;
            c.stage_bytes = sz;
        }
        char *db = (char *)c.d_stage;
        char *hb = pinned && c.h_stage ? (char *)c.h_stage : nullptr;
        if (hb) {
            memcpy(hb, in + j.lo, m * 8);
            if (hipMemcpyAsync(db, hb, m * 8, hipMemcpyHostToDevice, c.stream) != hipSuccess) return MK_EDEVICE;
        } else if (hipMemcpyAsync(db, in + j.lo, m * 8, hipMemcpyHostToDevice, c.stream) != hipSuccess) {
            return MK_EDEVICE;
        }
        mk_input mi{};
        mi.kind = MK_IN_I64;
        mi.data = db;
        rc = mk::launch_locked(h, j.d, &mi, m, (int32_t *)(db + a8), (uint8_t *)(db + a8 + a4 + a4),
                               steps ? (uint32_t *)(db + a8 + a4) : nullptr, nullptr, opts, c.stream);
        if (rc) return rc;
        char *o = hb ? hb + a8 : (char *)(out + j.lo);
        char *st = hb ? hb + a8 + a4 + a4 : (char *)(status + j.lo);
        char *sp = hb ? hb + a8 + a4 : (char *)(steps ? steps + j.lo : nullptr);
        if (hipMemcpyAsync(o, db + a8, m * 4, hipMemcpyDeviceToHost, c.stream) != hipSuccess ||
            hipMemcpyAsync(st, db + a8 + a4 + a4, m, hipMemcpyDeviceToHost, c.stream) != hipSuccess)
            return MK_EDEVICE;
        if (steps && hipMemcpyAsync(sp, db + a8 + a4, m * 4, hipMemcpyDeviceToHost, c.stream) != hipSuccess)
            return MK_EDEVICE;
    }
    int rc = MK_OK;
    for (auto &j : jobs) { // drain every device, then copy pinned results out
        mk::DevCtx &c = h->dev[j.d];
        mk::DeviceGuard g(j.d);
        if (hipStreamSynchronize(c.stream) != hipSuccess) {
            rc = MK_EDEVICE;
            continue;
        }
        const size_t m = j.hi - j.lo;
        if (m <= h->host_chunk && c.h_stage) {
            const char *hb = (const char *)c.h_stage;
            const size_t a8 = al(m * 8), a4 = al(m * 4);
            memcpy(out + j.lo, hb + a8, m * 4);
            if (steps) memcpy(steps + j.lo, hb + a8 + a4, m * 4);
            memcpy(status + j.lo, hb + a8 + a4 + a4, m);
        }
    }
    return rc;
}

int mk_compute_device(mk_net *h, int device, const mk_input *in, size_t n, int32_t *d_out, uint8_t *d_status,
                      uint32_t *d_steps, uint64_t *d_stats, const mk_opts *opts, void *stream)
{
    if (!h || !in || (n && (!d_out || !d_status))) return MK_EINVAL;
    if (in->kind != MK_IN_GEN && n && !in->data) return MK_EINVAL;
    if (in->kind < MK_IN_I64 || in->kind > MK_IN_GEN) return MK_EINVAL;
    const int ndev = mk::device_count();
    if (ndev <= 0) return MK_EDEVICE;
    if (device < 0 || device >= ndev || device >= mk::kMaxDevices) return MK_EINVAL;
    std::lock_guard<std::mutex> lk(h->mu);
    return mk::launch_locked(h, device, in, n, d_out, d_status, d_steps, d_stats, opts, (hipStream_t)stream);
}

int mk_session_create(mk_net *h, int device, size_t n, const mk_opts *opts, mk_session **out)
{
    if (!h || !out) return MK_EINVAL;
    *out = nullptr;
    const int ndev = mk::device_count();
    if (ndev <= 0) return MK_EDEVICE;
    if (device < 0 || device >= ndev || device >= mk::kMaxDevices) return MK_EINVAL;
    uint32_t budget, cap, flags;
    mk::resolve_opts(opts, budget, cap, flags);
    std::unique_ptr<mk_session> s(new (std::nothrow) mk_session());
    if (!s) return MK_ENOMEM;
    s->h = h;
    s->device = device;
    s->n = n;
    s->budget = budget;
    s->cap = cap;
    {
        std::lock_guard<std::mutex> lk(h->mu);
        int rc = mk::ensure_device(h, device);
        if (rc) return rc;
        s->nprog = h->net.nprog;
        // remote peers of a mixed deployment may push to / pop from local stacks
        s->nstack = h->net.uses_stacks || h->net.uses_remote ? h->net.nstack : 0;
    }
    mk::DeviceGuard g(device);
    // one allocation, 256-byte aligned arrays, [field][session]
    const size_t N = n ? n : 1, P = (size_t)s->nprog, S = (size_t)s->nstack;
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t sz[] = {al(P * N * 8), al(P * N * 8), al(P * N * 4), al(P * N * 4), al(P * 4 * N * 4), al(N * 8),
                         al(N * 4),     al(N * 4),     al(N * 4),     al(N * 4),     al(S * N * 4),     al(S * cap * N * 4),
                         al(P * N * 4), al(P * N * 4), al(N * 4),     al(N * 4)};
    size_t total = 0;
    for (size_t b : sz) total += b;
    if (hipMalloc(&s->d_state, total) != hipSuccess) return MK_ENOMEM;
    s->state_bytes = total;
    char *b = (char *)s->d_state;
    size_t off = 0;
    auto take = [&](size_t i) { char *q = b + off; off += sz[i]; return q; };
    mk::SessParams &p = s->p;
    for (int i = 0; i < s->nprog; i++) {
        p.base[i] = h->net.base[i];
        p.len[i] = h->net.len[i];
    }
    p.nprog = s->nprog;
    p.nstack = s->nstack;
    p.n = n;
    p.budget = budget;
    p.stack_cap = cap;
    p.acc = (int64_t *)take(0);
    p.bak = (int64_t *)take(1);
    p.ip = (int32_t *)take(2);
    p.pendv = (int32_t *)take(3);
    p.port = (int32_t *)take(4);
    p.pfull = (uint64_t *)take(5);
    p.bits = (uint32_t *)take(6);
    p.io = (uint32_t *)take(7);
    p.in_val = (int32_t *)take(8);
    p.out_val = (int32_t *)take(9);
    p.sdepth = (int32_t *)take(10);
    p.stk = (int32_t *)take(11);
    p.xst = (uint32_t *)take(12);
    p.xval = (int32_t *)take(13);
    p.pin = (int32_t *)take(14);
    p.csteps = (uint32_t *)take(15);
    p.mixed = h->net.uses_remote ? 1u : 0u;
    if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) return MK_EDEVICE;
    if (hipMemsetAsync(s->d_state, 0, total, s->stream) != hipSuccess) return MK_EDEVICE; // post-/reset state
    int rc = mk::session_native(s.get());
    if (rc) return rc;
    if (s->native_bytes && hipMemsetAsync(s->d_native, 0, s->native_bytes, s->stream) != hipSuccess)
        return MK_EDEVICE; // every session at the session schedule's first variant
    if (hipStreamSynchronize(s->stream) != hipSuccess) return MK_EDEVICE;
    *out = s.release();
    return MK_OK;
}

namespace mk {
// Orders work about to be queued on `to` after the session's last launch on
// a caller stream: a device-side wait on the event recorded after that
// launch, skipped when `to` is that same stream (stream order already holds;
// the two-way event hand-off per call had cost ~20 us of stream latency per
// launch, profiles/r06s_sessions_stream_order.txt).
int session_wait_last(mk_session *s, hipStream_t to)
{
    if (!s->last || s->last == to) return MK_OK;
    if (hipStreamWaitEvent(to, s->order, 0) != hipSuccess) return MK_EDEVICE;
    if (to == s->stream) s->last = nullptr; // s->stream now follows every launch so far
    return MK_OK;
}

// After a launch on `st` (a caller's or the session's own stream): work queued
// later on any other stream waits on this.
int session_mark(mk_session *s, hipStream_t st)
{
    if (!s->order && hipEventCreateWithFlags(&s->order, hipEventDisableTiming) != hipSuccess) return MK_EDEVICE;
    if (hipEventRecord(s->order, st) != hipSuccess) return MK_EDEVICE;
    s->last = st;
    return MK_OK;
}
} // namespace mk

int mk_session_reset(mk_session *s)
{
    if (!s) return MK_EINVAL;
    std::lock_guard<std::mutex> lk(s->mu);
    mk::DeviceGuard g(s->device);
    if (int rc = mk::session_wait_last(s, s->stream)) return rc;
    if (hipMemsetAsync(s->d_state, 0, s->state_bytes, s->stream) != hipSuccess) return MK_EDEVICE;
    if (s->native && hipMemsetAsync(s->d_native, 0, s->native_bytes, s->stream) != hipSuccess) return MK_EDEVICE;
    if (hipStreamSynchronize(s->stream) != hipSuccess) return MK_EDEVICE;
    s->broken = false; // every session back to its initial state, none handed off
    return MK_OK;
}

int mk_session_compute_seq_device(mk_session *s, const int64_t *d_in, size_t ncalls, int32_t *d_out,
                                  uint8_t *d_status, uint32_t *d_steps, void *stream)
{
    if (!s || (s->n && ncalls && (!d_in || !d_out || !d_status))) return MK_EINVAL;
    if (ncalls > 0xffffffffull) return MK_EINVAL;
    std::lock_guard<std::mutex> lk(s->mu);
    mk::DeviceGuard g(s->device);
    hipStream_t st = stream ? (hipStream_t)stream : s->stream;
    // the session state is ordered across streams device-side, with no host
    // synchronisation: this launch after the previous one (a wait only when
    // that ran on another stream), and the session's own stream's later work
    // (reset, host calls) after this one
    if (int rc = mk::session_wait_last(s, st)) return rc;
    bool queued = false;
    if (!s->order && hipEventCreateWithFlags(&s->order, hipEventDisableTiming) != hipSuccess) return MK_EDEVICE;
    int rc = mk::session_launch(s, d_in, d_out, d_status, d_steps, st, (uint32_t)ncalls, false, &queued, s->order);
    if (rc) {
        // the native kernel may be running on `st` although the launch
        // failed after it: reset and teardown must still wait for it
        if (queued) (void)mk::session_mark(s, st);
        return rc;
    }
    s->last = st; // the launch's last kernel recorded s->order (session_mark's event) on completion
    return MK_OK;
}

int mk_session_compute_device(mk_session *s, const int64_t *d_in, int32_t *d_out, uint8_t *d_status,
                              uint32_t *d_steps, void *stream)
{
    return mk_session_compute_seq_device(s, d_in, 1, d_out, d_status, d_steps, stream);
}

extern "C++" {
namespace mk {
namespace {
int session_host_calls(mk_session *s, const int64_t *in, size_t ncalls, int32_t *out, uint8_t *status,
                       uint32_t *steps, bool resume);
}
} // namespace mk
}

int mk_session_compute_seq(mk_session *s, const int64_t *in, size_t ncalls, int32_t *out, uint8_t *status,
                           uint32_t *steps)
{
    if (!s || (s->n && ncalls && (!in || !out || !status))) return MK_EINVAL;
    return mk::session_host_calls(s, in, ncalls, out, status, steps, false);
}

int mk_session_step(mk_session *s, const int64_t *in, int32_t *out, uint8_t *status, uint32_t *steps)
{
    if (!s || (s->n && (!out || !status))) return MK_EINVAL;
    if (!in) { // resume: the kernel ignores the inputs
        std::vector<int64_t> z(s->n ? s->n : 1, 0);
        return mk::session_host_calls(s, z.data(), 1, out, status, steps, true);
    }
    return mk::session_host_calls(s, in, 1, out, status, steps, false);
}

extern "C++" {
namespace mk {
namespace {
int session_host_calls(mk_session *s, const int64_t *in, size_t ncalls, int32_t *out, uint8_t *status,
                       uint32_t *steps, bool resume)
{
    if (s->n == 0 || ncalls == 0) return MK_OK;
    if (ncalls > 0xffffffffull) return MK_EINVAL;
    std::lock_guard<std::mutex> lk(s->mu);
    mk::DeviceGuard g(s->device);
    if (int rc = mk::session_wait_last(s, s->stream)) return rc;
    const size_t m = s->n * ncalls;
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t a8 = al(m * 8), a4 = al(m * 4), need = a8 + a4 + a4 + al(m);
    // device buffers plus a pinned host mirror (small bursts are latency-bound:
    // pinned copies avoid the runtime's pageable staging and its extra sync)
    if (need > s->stage_bytes) {
        (void)hipFree(s->d_stage);
        (void)hipHostFree(s->h_stage);
        s->d_stage = s->h_stage = nullptr;
        s->stage_bytes = 0;
        if (hipMalloc(&s->d_stage, need) != hipSuccess) return MK_ENOMEM;
        if (hipHostMalloc(&s->h_stage, need, hipHostMallocDefault) != hipSuccess) return MK_ENOMEM;
        s->stage_bytes = need;
    }
    char *b = (char *)s->d_stage, *hb = (char *)s->h_stage;
    int64_t *din = (int64_t *)b;
    int32_t *dout = (int32_t *)(b + a8);
    uint32_t *dsteps = (uint32_t *)(b + a8 + a4);
    uint8_t *dst = (uint8_t *)(b + a8 + a4 + a4);
    memcpy(hb, in, m * 8);
    if (hipMemcpyAsync(din, hb, m * 8, hipMemcpyHostToDevice, s->stream) != hipSuccess) return MK_EDEVICE;
    int rc = mk::session_launch(s, din, dout, dst, steps ? dsteps : nullptr, s->stream, (uint32_t)ncalls, resume);
    if (rc) return rc;
    if (hipMemcpyAsync(hb + a8, dout, m * 4, hipMemcpyDeviceToHost, s->stream) != hipSuccess ||
        hipMemcpyAsync(hb + a8 + a4 + a4, dst, m, hipMemcpyDeviceToHost, s->stream) != hipSuccess)
        return MK_EDEVICE;
    if (steps && hipMemcpyAsync(hb + a8 + a4, dsteps, m * 4, hipMemcpyDeviceToHost, s->stream) != hipSuccess)
        return MK_EDEVICE;
    if (hipStreamSynchronize(s->stream) != hipSuccess) return MK_EDEVICE;
    memcpy(out, hb + a8, m * 4);
    memcpy(status, hb + a8 + a4 + a4, m);
    if (steps) memcpy(steps, hb + a8 + a4, m * 4);
    // a session that had a call open when this launch began did nothing
    // (MK_ST_CALL_OPEN): resume or cancel that call first
    if (!resume)
        for (size_t i = 0; i < s->n; i++)
            if (status[i] == MK_ST_CALL_OPEN) return MK_EBUSY;
    return MK_OK;
}

// One element of session state (device), read or written synchronously on
// the session's stream (ordered after its launches).  Caller holds s->mu.
template <class T>
int sget(mk_session *s, const T *dev, T &v)
{
    if (int rc = session_wait_last(s, s->stream)) return rc;
    if (hipMemcpyAsync(&v, dev, sizeof(T), hipMemcpyDeviceToHost, s->stream) != hipSuccess) return MK_EDEVICE;
    return hipStreamSynchronize(s->stream) == hipSuccess ? MK_OK : MK_EDEVICE;
}
template <class T>
int sput(mk_session *s, T *dev, const T &v)
{
    if (int rc = session_wait_last(s, s->stream)) return rc;
    if (hipMemcpyAsync(dev, &v, sizeof(T), hipMemcpyHostToDevice, s->stream) != hipSuccess) return MK_EDEVICE;
    return hipStreamSynchronize(s->stream) == hipSuccess ? MK_OK : MK_EDEVICE;
}
} // namespace
} // namespace mk
}

int mk_session_compute(mk_session *s, const int64_t *in, int32_t *out, uint8_t *status, uint32_t *steps)
{
    return mk_session_compute_seq(s, in, 1, out, status, steps);
}

int mk_session_remote_poll(mk_session *s, size_t inst, mk_remote_req *reqs, int max, int *count)
{
    if (!s || !count || inst >= s->n || (max > 0 && !reqs)) return MK_EINVAL;
    std::lock_guard<std::mutex> lk(s->mu);
    mk::DeviceGuard g(s->device);
    *count = 0;
    if (!s->p.mixed) return MK_OK;
    const uint64_t n = s->n;
    for (int k = 0; k < s->nprog; k++) {
        uint32_t st = 0;
        int rc = mk::sget(s, s->p.xst + (uint64_t)k * n + inst, st);
        if (rc) return rc;
        if (st != 1u) continue;
        int32_t ip = 0, val = 0;
        if ((rc = mk::sget(s, s->p.ip + (uint64_t)k * n + inst, ip)) ||
            (rc = mk::sget(s, s->p.xval + (uint64_t)k * n + inst, val)))
            return rc;
        const mk::Insn &I = s->h->net.code[s->h->net.base[k] + (uint32_t)ip];
        if (*count >= max) return MK_EINVAL;
        mk_remote_req &r = reqs[(*count)++];
        r.node = (uint32_t)k;
        r.op = I.op == mk::OP_XSEND ? MK_REMOTE_SEND : I.op == mk::OP_XPUSH ? MK_REMOTE_PUSH : MK_REMOTE_POP;
        r.remote = I.op == mk::OP_XSEND ? I.arg / 4u : I.arg;
        r.reg = I.op == mk::OP_XSEND ? I.arg % 4u : 0u;
        r.value = val;
    }
    return MK_OK;
}

int mk_session_remote_done(mk_session *s, size_t inst, uint32_t node, int32_t value)
{
    if (!s || inst >= s->n || node >= (uint32_t)s->nprog || !s->p.mixed) return MK_EINVAL;
    std::lock_guard<std::mutex> lk(s->mu);
    mk::DeviceGuard g(s->device);
    const uint64_t off = (uint64_t)node * s->n + inst;
    uint32_t st = 0;
    int rc = mk::sget(s, s->p.xst + off, st);
    if (rc) return rc;
    if (st != 1u) return MK_EINVAL; // no request outstanding
    if ((rc = mk::sput(s, s->p.xval + off, value))) return rc;
    return mk::sput(s, s->p.xst + off, (uint32_t)2u);
}

int mk_session_port_put(mk_session *s, size_t inst, uint32_t node, uint32_t reg, int32_t value)
{
    if (!s || inst >= s->n || node >= (uint32_t)s->nprog || reg > 3) return MK_EINVAL;
    if (s->native) return MK_EINVAL; // host-side state access: interpreter sessions (mixed networks) only
    std::lock_guard<std::mutex> lk(s->mu);
    mk::DeviceGuard g(s->device);
    const uint32_t q = node * 4 + reg;
    uint64_t full = 0;
    int rc = mk::sget(s, s->p.pfull + inst, full);
    if (rc) return rc;
    if ((full >> q) & 1ull) return MK_EBUSY; // p.rK <- v blocks while full (program.go:163)
    if ((rc = mk::sput(s, s->p.port + (uint64_t)q * s->n + inst, value))) return rc;
    return mk::sput(s, s->p.pfull + inst, (uint64_t)(full | (1ull << q)));
}

int mk_session_stack_push(mk_session *s, size_t inst, uint32_t stack, int32_t value)
{
    if (!s || inst >= s->n || stack >= (uint32_t)s->nstack) return MK_EINVAL;
    if (s->native) return MK_EINVAL; // host-side state access: interpreter sessions (mixed networks) only
    std::lock_guard<std::mutex> lk(s->mu);
    mk::DeviceGuard g(s->device);
    int32_t d = 0;
    int rc = mk::sget(s, s->p.sdepth + (uint64_t)stack * s->n + inst, d);
    if (rc) return rc;
    if ((uint32_t)d >= s->cap) return MK_ELIMIT; // stack_cap (the reference's stacks are unbounded)
    if ((rc = mk::sput(s, s->p.stk + ((uint64_t)stack * s->cap + (uint32_t)d) * s->n + inst, value))) return rc;
    return mk::sput(s, s->p.sdepth + (uint64_t)stack * s->n + inst, (int32_t)(d + 1));
}

int mk_session_stack_pop(mk_session *s, size_t inst, uint32_t stack, int32_t *value)
{
    if (!s || !value || inst >= s->n || stack >= (uint32_t)s->nstack) return MK_EINVAL;
    if (s->native) return MK_EINVAL; // host-side state access: interpreter sessions (mixed networks) only
    std::lock_guard<std::mutex> lk(s->mu);
    mk::DeviceGuard g(s->device);
    int32_t d = 0;
    int rc = mk::sget(s, s->p.sdepth + (uint64_t)stack * s->n + inst, d);
    if (rc) return rc;
    if (d <= 0) return MK_EBUSY; // waitPop blocks while empty (stack.go:133-155)
    if ((rc = mk::sget(s, s->p.stk + ((uint64_t)stack * s->cap + (uint32_t)(d - 1)) * s->n + inst, *value)))
        return rc;
    return mk::sput(s, s->p.sdepth + (uint64_t)stack * s->n + inst, (int32_t)(d - 1));
}

int mk_session_input_take(mk_session *s, size_t inst, int32_t *value)
{
    if (!s || !value || inst >= s->n) return MK_EINVAL;
    if (s->native) return MK_EINVAL; // host-side state access: interpreter sessions (mixed networks) only
    std::lock_guard<std::mutex> lk(s->mu);
    mk::DeviceGuard g(s->device);
    uint32_t io = 0;
    int rc = mk::sget(s, s->p.io + inst, io);
    if (rc) return rc;
    if (io & 1u) { // <-m.inChan (master.go:235)
        if ((rc = mk::sget(s, s->p.in_val + inst, *value))) return rc;
        return mk::sput(s, s->p.io + inst, io & ~1u);
    }
    if ((io & 0xCu) == 0xCu) // the open call is still waiting to deposit (m.inChan <- v, :216): hand it over
        return (rc = mk::sget(s, s->p.pin + inst, *value)) ? rc : mk::sput(s, s->p.io + inst, io & ~4u);
    return MK_EBUSY; // GetInput blocks while inChan is empty
}

int mk_session_output_put(mk_session *s, size_t inst, int32_t value)
{
    if (!s || inst >= s->n) return MK_EINVAL;
    if (s->native) return MK_EINVAL; // host-side state access: interpreter sessions (mixed networks) only
    std::lock_guard<std::mutex> lk(s->mu);
    mk::DeviceGuard g(s->device);
    uint32_t io = 0;
    int rc = mk::sget(s, s->p.io + inst, io);
    if (rc) return rc;
    if (io & 2u) return MK_EBUSY; // m.outChan <- v blocks while full (master.go:246)
    if ((rc = mk::sput(s, s->p.out_val + inst, value))) return rc;
    return mk::sput(s, s->p.io + inst, io | 2u);
}

int mk_net_node_index(const mk_net *h, const char *name, int *kind, int *index)
{
    if (!h || !name || !kind || !index) return MK_EINVAL;
    const mk::Network &N = h->net;
    for (int i = 0; i < N.nprog; i++)
        if (N.prog_names[i] == name) { *kind = MK_NODE_PROGRAM; *index = i; return MK_OK; }
    for (int i = 0; i < N.nstack; i++)
        if (N.stack_names[i] == name) { *kind = MK_NODE_STACK; *index = i; return MK_OK; }
    for (size_t i = 0; i < N.remote_names.size(); i++)
        if (N.remote_names[i] == name) { *kind = N.remote_kinds[i]; *index = (int)i; return MK_OK; }
    return MK_EINVAL;
}

int mk_session_cancel(mk_session *s)
{
    if (!s) return MK_EINVAL;
    if (s->n == 0) return MK_OK;
    std::lock_guard<std::mutex> lk(s->mu);
    mk::DeviceGuard g(s->device);
    if (int rc = mk::session_wait_last(s, s->stream)) return rc;
    uint32_t *io = s->p.io;
    uint64_t n = s->n;
    void *args[] = {(void *)&io, (void *)&n};
    const uint64_t blocks = (n + mk::kBlock - 1) / mk::kBlock;
    if (hipLaunchKernel(reinterpret_cast<void *>(&mk::tis_session_cancel), dim3((unsigned)blocks), dim3(mk::kBlock),
                        args, 0, s->stream) != hipSuccess)
        return MK_EDEVICE;
    return hipStreamSynchronize(s->stream) == hipSuccess ? MK_OK : MK_EDEVICE;
}

int mk_session_plan(const mk_session *s, char *out, size_t out_len)
{
    if (!s) return MK_EINVAL;
    return mk::copy_out(out, out_len, s->plan);
}

void mk_session_free(mk_session *s) { delete s; }

int mk_trace_lane(mk_net *h, int device, int64_t input, const mk_opts *opts, mk_trace_entry *out,
                  uint32_t max_entries, uint32_t *count, uint8_t *status)
{
    if (!h || !count || !status || (max_entries && !out)) return MK_EINVAL;
    const int ndev = mk::device_count();
    if (ndev <= 0) return MK_EDEVICE;
    if (device < 0 || device >= ndev || device >= mk::kMaxDevices) return MK_EINVAL;
    std::lock_guard<std::mutex> lk(h->mu);
    int rc = mk::ensure_device(h, device);
    if (rc) return rc;
    mk::DevCtx &c = h->dev[device];
    mk::DeviceGuard g(device);
    // one lane on the bytecode interpreter (tier 1), the only tier that
    // executes one TIS instruction at a time
    mk_opts o{};
    if (opts) o = *opts;
    o.flags = (o.flags & MK_FLAG_STOP_ON_OUTPUT) | MK_FLAG_FORCE_INTERP;
    const size_t tb = (size_t)max_entries * sizeof(mk_trace_entry);
    char *buf = nullptr;
    if (hipMalloc(&buf, 256 + tb + 64) != hipSuccess) return MK_ENOMEM;
    int64_t *din = (int64_t *)buf;
    int32_t *dout = (int32_t *)(buf + 8);
    uint8_t *dst = (uint8_t *)(buf + 12);
    uint32_t *dn = (uint32_t *)(buf + 16);
    mk_trace_entry *dtr = (mk_trace_entry *)(buf + 256);
    mk_input mi{};
    mi.kind = MK_IN_I64;
    mi.data = din;
    if (hipMemcpyAsync(din, &input, 8, hipMemcpyHostToDevice, c.stream) != hipSuccess ||
        hipMemsetAsync(dn, 0, 4, c.stream) != hipSuccess)
        rc = MK_EDEVICE;
    if (!rc) rc = mk::launch_locked(h, device, &mi, 1, dout, dst, nullptr, nullptr, &o, c.stream, dtr, max_entries, dn);
    if (!rc && (hipMemcpyAsync(count, dn, 4, hipMemcpyDeviceToHost, c.stream) != hipSuccess ||
                hipMemcpyAsync(status, dst, 1, hipMemcpyDeviceToHost, c.stream) != hipSuccess ||
                hipStreamSynchronize(c.stream) != hipSuccess))
        rc = MK_EDEVICE;
    if (!rc && *count && hipMemcpy(out, dtr, (size_t)*count * sizeof(mk_trace_entry), hipMemcpyDeviceToHost) != hipSuccess)
        rc = MK_EDEVICE;
    (void)hipFree(buf);
    return rc;
}

int mk_stats_fold(mk_net *h, int device, uint64_t *d_stats, void *stream)
{
    if (!h || !d_stats) return MK_EINVAL;
    const int ndev = mk::device_count();
    if (ndev <= 0) return MK_EDEVICE;
    if (device < 0 || device >= ndev || device >= mk::kMaxDevices) return MK_EINVAL;
    std::lock_guard<std::mutex> lk(h->mu);
    int rc = mk::ensure_device(h, device);
    if (rc) return rc;
    mk::DevCtx &c = h->dev[device];
    mk::DeviceGuard g(device);
    if ((rc = mk::order_on(c, (hipStream_t)stream))) return rc;
    if ((rc = mk::ensure_partials(c, 0))) return rc;
    return mk::launch_stats_reduce(c, d_stats, (hipStream_t)stream);
}

int mk_generate_inputs_device(int device, uint64_t seed, uint32_t gen_kind, uint32_t gen_mask, uint64_t offset,
                              size_t n, int32_t *d_out, void *stream)
{
    if (n == 0) return MK_OK;
    if (!d_out) return MK_EINVAL;
    const int ndev = mk::device_count();
    if (ndev <= 0) return MK_EDEVICE;
    if (device < 0 || device >= ndev) return MK_EINVAL;
    mk::DeviceGuard g(device);
    const uint64_t blocks = std::min<uint64_t>((n + mk::kBlock - 1) / mk::kBlock, 8192);
    hipLaunchKernelGGL(mk::gen_inputs, dim3((unsigned)blocks), dim3(mk::kBlock), 0, (hipStream_t)stream, seed,
                       gen_kind, gen_mask, offset, (uint64_t)n, d_out);
    return hipGetLastError() == hipSuccess ? MK_OK : MK_EDEVICE;
}

int mk_valu_probe_device(int device, int blocks, int iters, uint64_t *lane_ops, void *stream)
{
    if (blocks <= 0 || iters <= 0) return MK_EINVAL;
    const int ndev = mk::device_count();
    if (ndev <= 0) return MK_EDEVICE;
    if (device < 0 || device >= ndev) return MK_EINVAL;
    mk::DeviceGuard g(device);
    static uint32_t *sink[mk::kMaxDevices] = {};
    static std::mutex smu;
    {
        std::lock_guard<std::mutex> lk(smu);
        if (!sink[device] && hipMalloc(&sink[device], 4) != hipSuccess) return MK_ENOMEM;
    }
    hipLaunchKernelGGL(mk::valu_probe, dim3(blocks), dim3(mk::kBlock), 0, (hipStream_t)stream, iters, sink[device]);
    if (lane_ops) *lane_ops = (uint64_t)blocks * mk::kBlock * (uint64_t)iters * 64u;
    return hipGetLastError() == hipSuccess ? MK_OK : MK_EDEVICE;
}

int mk_tokenize(const char *program, char *out, size_t out_len)
{
    if (!program || !out || !out_len) return MK_EINVAL;
    mk::Program P;
    std::string err;
    if (!mk::parse_program(program, P, err)) {
        mk::set_err(out, out_len, err);
        return MK_EPARSE;
    }
    std::string s;
    for (size_t i = 0; i < P.lines.size(); i++) {
        if (i) s += '\n';
        s += mk::form_name(P.lines[i].form);
        if (!P.lines[i].a.empty()) { s += '\x1f'; s += P.lines[i].a; }
        if (!P.lines[i].b.empty()) { s += '\x1f'; s += P.lines[i].b; }
    }
    return mk::copy_out(out, out_len, s);
}

int mk_net_disasm(const mk_net *net, char *out, size_t out_len)
{
    if (!net) return MK_EINVAL;
    return mk::copy_out(out, out_len, mk::disasm(net->net));
}

int mk_net_plan(mk_net *h, const mk_opts *opts, char *out, size_t out_len)
{
    if (!h) return MK_EINVAL;
    uint32_t budget, cap, flags;
    mk::resolve_opts(opts, budget, cap, flags);
    char buf[1024];
    std::lock_guard<std::mutex> lk(h->mu);
    mk::SchedCache *sc = nullptr;
    const mk::Tier t = mk::pick_tier(h, cap, flags, budget, &sc);
    if (t == mk::TIER_INTERP) {
        if (sc && sc->ok)
            snprintf(buf, sizeof buf, "tier=interp reason=compiled schedule of %u superblocks (control state follows "
                     "the data); native tier: %s", mk::tier2_prog(sc).nsb, sc->jit.why.c_str());
        else
            snprintf(buf, sizeof buf, "tier=interp reason=%s", sc ? sc->why.c_str() : "forced");
        return mk::copy_out(out, out_len, buf);
    }
    if (t == mk::TIER_NONE) {
        snprintf(buf, sizeof buf, "tier=none reason=native tier unavailable: %s",
                 sc->jit.ok ? "budget within the network's longest path (the native stream kernel has no budget checks)"
                            : sc->jit.why.c_str());
        (void)mk::copy_out(out, out_len, buf);
        return MK_ELIMIT;
    }
    // the native tier's schedule, or tier 2's (the default plan)
    const mk::SchedProgram &P = t == mk::TIER_NATIVE ? sc->prog : mk::tier2_prog(sc);
    int len = snprintf(buf, sizeof buf, "superblocks=%u regs=%u slots=%u words=%zu jtab=%zu rounds=%llu", P.nsb,
                       P.nregs, P.nslots, P.code.size(), P.jtab.size(), (unsigned long long)P.sym_rounds);
    std::string s;
    if (t == mk::TIER_NATIVE) {
        char tail[200];
        snprintf(tail, sizeof tail, " shape=%s%s source=%zuB kernel=%016llx code=%zuB compile=%.2fs rtc=%s",
                 sc->jit.shape == mk::JIT_MACHINE ? "machine"
                 : sc->jit.heavy                  ? (sc->jit.lds ? "stream-heavy-lds"
                                                     : sc->jit.lds_n ? "stream-heavy-split"
                                                                     : "stream-heavy")
                                                  : "stream",
                 sc->jit.pool >= 64 ? ("-pool" + std::to_string(sc->jit.pool)).c_str()
                 : sc->jit.pool     ? ("-k" + std::to_string(sc->jit.pool)).c_str()
                                    : "",
                 sc->jit.src_bytes, (unsigned long long)sc->jit.src_hash,
                 sc->jit.code.size(), sc->jit.compile_s, sc->jit.rtc.c_str());
        s = std::string("tier=native ") + buf + tail;
        if (sc->jit.rtc == "linked-other") { // the namespace compiler was wanted but could not open
            std::string r = mk::ns_fail_reason();
            if (!r.empty()) {
                std::replace(r.begin(), r.end(), ' ', '_');
                s += " rtc_ns_error=" + r;
            }
        }
        // heavy kernel, slots in HBM: at most this many inputs per launch
        // (the slot memory cap, JitLimits::slot_bytes; launch_jit_locked)
        const uint32_t hbm_slots = P.nslots - sc->jit.lds_n;
        if (sc->jit.shape == mk::JIT_STREAM && sc->jit.heavy && hbm_slots) {
            const uint64_t blk = (uint64_t)sc->jit.block, fit = h->jit_lim.slot_bytes / ((uint64_t)hbm_slots * 4u);
            s += " chunk=" + std::to_string(std::max<uint64_t>(blk, fit / blk * blk));
        }
        if (!sc->occ_note.empty()) s += " stack_plans=" + sc->occ_note; // more_waves: what the checks found
        s += " knobs=" + h->jit_lim.key();
        // resident waves per SIMD of the loaded kernel (registers and LDS;
        // the first device it is loaded on): the occupancy its issue rate is
        // priced at (bench.py roofline_issue.occupancy)
        // (a fraction when the blocks per CU do not fill the four SIMDs
        // evenly: 15 blocks of one wave are 3.75 per SIMD, not 3)
        for (int d = 0; d < mk::kMaxDevices; d++)
            if (sc->jit.dev[d].fn) {
                // (the last launch's grid when it held fewer blocks than the
                // resident grid: a small batch, or GridTune's choice)
                const mk::JitDev &jd = sc->jit.dev[d];
                const int cus = std::max(h->dev[d].cus, 1);
                const double bcu = jd.last_blocks > 0 && jd.last_blocks < jd.per_cu * cus
                                       ? (double)jd.last_blocks / cus : (double)jd.per_cu;
                const double wps = bcu * sc->jit.block / 64 / 4; // waves per SIMD
                char w[32];
                if (wps == (double)(int)wps) snprintf(w, sizeof w, "%d", (int)wps);
                else snprintf(w, sizeof w, "%.2f", wps);
                s += std::string(" waves_per_simd=") + w;
                // GridTune's choice for the last tuned batch size (blocks of
                // the resident grid's), once measured
                const int tl = jd.tune_last;
                const mk::GridTune &t = jd.tune[tl < 0 ? 0 : tl];
                if (tl >= 0 && t.phase == 4 && t.cand[2])
                    s += " grid_tuned=" + std::to_string(t.chosen) + "/" + std::to_string(t.cand[2]);
                break;
            }
    } else {
        const bool tile = (flags & MK_FLAG_TILE) ? true : (flags & MK_FLAG_REFILL) ? false : sc->tile;
        uint32_t B, K;
        mk::sched_geometry(P.nregs, B, K);
        snprintf(buf + len, sizeof buf - len, " lanes=%s K=%u B=%u native=%s", tile ? "tile" : "refill", K, B,
                 !sc->jit.tried ? "not-requested"
                 : !sc->jit.ok  ? sc->jit.why.c_str()
                                : "ok-but-budget-within-longest-path");
        s = std::string("tier=compiled ") + buf;
    }
    return mk::copy_out(out, out_len, s);
}

int mk_net_prepare(mk_net *h, const mk_opts *opts, int device)
{
    if (!h || device < 0 || device >= mk::kMaxDevices) return MK_EINVAL;
    uint32_t budget, cap, flags;
    mk::resolve_opts(opts, budget, cap, flags);
    std::lock_guard<std::mutex> lk(h->mu);
    int rc = mk::ensure_device(h, device);
    if (rc) return rc;
    mk::SchedCache *sc = nullptr;
    switch (mk::pick_tier(h, cap, flags, budget, &sc)) {
    case mk::TIER_NATIVE: return mk::ensure_jit_device(sc, device);
    case mk::TIER_COMPILED: return mk::ensure_sched_device(sc, device);
    case mk::TIER_NONE: return MK_ELIMIT;
    default: return MK_OK;
    }
}

int mk_net_jit_source(mk_net *h, const mk_opts *opts, char *out, size_t out_len)
{
    if (!h) return MK_EINVAL;
    uint32_t budget, cap, flags;
    mk::resolve_opts(opts, budget, cap, flags);
    std::lock_guard<std::mutex> lk(h->mu);
    mk::SchedCache *sc = mk::get_sched(h, cap, (flags & MK_FLAG_STOP_ON_OUTPUT) != 0);
    std::string lane, why;
    if (!sc->ok) why = sc->why;
    else {
        mk::JitShape shape;
        bool heavy = false;
        uint32_t pool = 0;
        mk::JitLimits L = h->jit_lim; // as jit_compile: the network's LDS budget
        if (sc->lds_set) L.lds_slot_bytes = sc->lds_bytes;
        if (sc->max_dops) L.max_dops = std::max(L.max_dops, sc->max_dops);
        if (mk::jit_lane_source(sc->prog, L, lane, why, &shape, nullptr, &heavy, false, &pool)) {
            if (shape == mk::JIT_MACHINE) L.ts_rounds = mk::jit_sort_rounds(L, sc->prog.nslots);
            return mk::copy_out(out, out_len, mk::jit_module_source(lane, shape, heavy && shape == mk::JIT_STREAM,
                                                                    L, pool));
        }
    }
    (void)mk::copy_out(out, out_len, why);
    return MK_ELIMIT;
}

int mk_net_sched_disasm(mk_net *h, const mk_opts *opts, char *out, size_t out_len)
{
    if (!h) return MK_EINVAL;
    uint32_t budget, cap, flags;
    mk::resolve_opts(opts, budget, cap, flags);
    std::lock_guard<std::mutex> lk(h->mu);
    mk::SchedCache *sc = mk::get_sched(h, cap, (flags & MK_FLAG_STOP_ON_OUTPUT) != 0);
    if (!sc->ok) return MK_ELIMIT;
    return mk::copy_out(out, out_len, mk::sched_disasm(mk::tier2_prog(sc)));
}

int mk_net_info(const mk_net *net, int *counts3)
{
    if (!net || !counts3) return MK_EINVAL;
    counts3[0] = net->net.nprog;
    counts3[1] = net->net.nstack;
    counts3[2] = (int)net->net.code.size();
    return MK_OK;
}

} // extern "C"
