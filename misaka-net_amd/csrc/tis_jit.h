// tis_jit.h -- tier 3: a network's compiled schedule (tis_sched.h) turned
// into native code, one kernel per (network, stack_cap, stop_on_output),
// compiled for gfx950 at run time by hiprtc.
//
// Superblock variants become code, their micro-ops int64 expressions on
// VGPR-resident variables (instead of the LDS register file of tier 2).
// Nothing is interpreted at run time: no fetch, no decode.  Two shapes:
//   JIT_STREAM  -- acyclic superblock graph (every lane runs a bounded
//                  straight-line path): labels + gotos in one lane function;
//                  the kernel streams 4 lanes per thread with vector I/O.
//   JIT_MACHINE -- cyclic graph (data-dependent loops): the lane is a
//                  resumable state machine (MkLane + mk_run per variant, self
//                  loops as rotated do-while loops); the kernel dispatches one
//                  superblock per wave turn and refills finished lanes with
//                  new inputs while the rest of the wave keeps running.
#pragma once

#include <cstdint>
#include <string>

#include "tis_sched.h"

namespace mk {

enum JitShape { JIT_STREAM = 0, JIT_MACHINE = 1 };

constexpr size_t kJitHeavyOps = 256; // stream lanes above this size: one lane per thread
// Heavy kernels run one thread per input; a launch covers at most as many
// inputs as fit this much stack-slot memory (more take several launches).
// 256 MiB: a launch's slot blocks stay in the 256 MB Infinity Cache, so the
// pushes and pops of a launch mostly never reach HBM (r03g/r03h, C4 D=1024
// at 256K lanes: 2.72 ms in one launch of 1 GB of slots; 2.30-2.43 ms in
// launches of 128-256 MiB, 2.55 at 320, 4.0 at 48 -- too few waves).
constexpr size_t kJitSlotBytes = size_t(256) << 20;
// Heavy stream kernel: stack slots in LDS up to this many bytes per wave
// (JitLimits::lds_slot_bytes): two waves per CU.  Measured on MI355X (r02x,
// r02an): C4 D=64 (41 shared slots, 10 KB per wave) 194 -> 59 us against its
// slots in HBM; D=256 (233 slots, 58 KB) 1.14 -> 0.61 ms; D=320 (297 slots,
// 74 KB) 738 -> 498 us; with one wave per CU HBM wins (D=400: 964 vs 1,098 us,
// D=500 and 640 likewise).
constexpr size_t kJitLdsSlotBytes = 81920;
// Default machine-shape policy word (kMachineKernel): generations -- a wave
// refills only once all its lanes have ended and loops never leave early.
// Measured on MI355X (C5): ahead of every early-refill / early-leave setting
// tried (refill 1..48 lanes, leave at 8..14/16), whose extra dispatches and
// small groups cost more than the idle lanes they save.
constexpr uint32_t kJitPolicy = 64u | (0u << 8) | (64u << 16);
// POP loops keep this many slot reads in flight (emit_prefetched_run).
constexpr size_t kJitPrefetchLoads = 16;

// Limits and code-shape knobs of the native tier.  The defaults are the
// product; from_env() overlays the MK_JIT_* experiment variables.  A loaded
// network takes one snapshot at mk_net_load, so every module it compiles,
// every plan it reports and every launch it makes use the same knobs (a
// later change of the environment affects networks loaded after it).
struct JitLimits {
    uint32_t max_variants = 4096; // superblock variants (labels)
    size_t max_dops = 4096;       // micro-ops emitted, after rolling repeats into loops
                                  // (hiprtc time grows superlinearly: 14K straight-line
                                  // ops take ~150 s)
    size_t max_scan = 1u << 22;   // micro-ops of reachable code scanned before giving up
    // Bound on the generated lane source handed to hiprtc (bytes, without the
    // host-only checked variant).  Compile time follows the size of the
    // function LLVM sees; past this the network stays on tier 2 with the
    // reason in mk_net_plan (MK_JIT_MAX_SRC).
    size_t max_src_bytes = size_t(1) << 20;
    // Wall-clock bound on one hiprtc compilation (seconds, MK_JIT_COMPILE_S):
    // the compile runs on a helper thread, and when it does not finish in
    // time the network stays on tier 2 (the compile is left to finish in the
    // background and its result discarded).
    double max_compile_s = 60.0;
    bool disabled = false;      // MK_JIT=0: no native tier
    bool force_machine = false; // MK_JIT_SHAPE=machine: machine shape even for acyclic graphs (tests)
    bool force_stream = false;  // MK_JIT_SHAPE=stream: stream shape even for cyclic graphs (experiments)
    uint32_t policy = kJitPolicy;          // MK_JIT_POLICY=refill,num,min
    int loop_unroll = 0;                   // MK_JIT_LOOP_UNROLL (0: by body size, fast_unroll)
    int slot_layout = -1;                  // MK_JIT_SLOT_LAYOUT=blocked(1)|lane(0); -1: by size
    size_t prefetch = kJitPrefetchLoads;   // MK_JIT_PREFETCH (0: off)
    size_t heavy_ops = kJitHeavyOps;       // MK_JIT_HEAVY_OPS
    uint64_t slot_bytes = kJitSlotBytes;   // MK_JIT_SLOT_BYTES
    // Lane compaction in the machine shape (experiments, MK_JIT_POOL):
    //   0     the pool-less kernel, generations (default: fastest measured);
    //   2..8  K lanes per thread in registers, swapped at loop heads
    //         (kMachineMultiKernel);
    //   >=64  an LDS pool of that many parked lanes per wave, largest-group
    //         dispatch (kMachinePoolKernel).
    // Both compaction kernels are bit-exact and slower on C5.
    uint32_t pool = 0;
    // Machine shape: run the inputs grouped by value (a counting sort of the
    // batch's indices before the launch), so that a wave's lanes have
    // similar loop trip counts (MK_JIT_ORDER=1).  Off by default: on C5 the
    // sort's contended bucket atomics and the scattered result writes cost
    // more than the idle lanes it saves (780 vs 367 us, r02g).
    bool order = false;
    // Machine shape: group the inputs by value inside each block's tile of
    // 1024 (an LDS counting sort, kMachineSortKernel) so that a wave's lanes
    // have similar loop trip counts (MK_JIT_TILE_SORT=0: input order).
    bool tile_sort = true;
    // Its tile: 256 x ts_rounds inputs, each wave running ts_rounds sorted
    // chunks of 64 per tile (MK_JIT_TS_ROUNDS = 4, 8 or 16).  r02v: 8 is 2%
    // faster on C5 (211 vs 215 us) but 20% / 8% slower on the dynamic-stack
    // census classes (twice the stack slots in flight per tile); 16 halves
    // the blocks per CU (61 KB of LDS) and loses everywhere.  0: 8 for
    // lanes without stack slots, 4 with them -- r02ak: C5 212-214 vs 215 us
    // but the JRO-heavy census class 58.9 vs 52.1 ms, so not the default.
    uint32_t ts_rounds = 4;
    // ... for lanes with stack slots (MK_JIT_TS_ROUNDS_SLOTS = 1, 2, 4, 8 or
    // 16; 0: as ts_rounds).  Round 6: tiles of 512 take the dynamic-stack
    // census classes to more waves per SIMD (2,048 tiles fill the resident
    // grid): t1_two_stacks 194 -> 182 us, t2_dyn_depth 119 -> 116 us; 256
    // loses (216 / 133 us) (profiles/r08_grid_tune_ab.txt, r08ap).
    uint32_t ts_rounds_slots = 2;
    // kMachineSortKernel dispatches by sweeps over the variants in reverse
    // postorder (tis_jit.cpp forward_order), each variant one ballot when no
    // lane is on it, instead of one variant per round (MK_JIT_SWEEP=0: rounds;
    // C5 105.8 -> 97.0 us, profiles/r06u_c5_sweep_ab.txt).
    bool sweep = true;
    // Heavy stream kernel: a lane's stack slots live in LDS instead of HBM
    // when the wave's nslots x 256 B fit this many bytes (MK_JIT_LDS_SLOTS,
    // 0 = never).  One 64-thread block per wave, so the bound also sets the
    // waves per CU the LDS allows (160 KiB / bytes).
    size_t lds_slot_bytes = kJitLdsSlotBytes;
    // The loader picks each heavy network's LDS budget and register count
    // (mk_exec.hip tune_soft_regs) unless MK_JIT_LDS_SLOTS sets the budget.
    bool lds_auto = true;
    // Machine-shape countdown loops (x > 0, x -= 1) run, past their first
    // iteration, as one saturating decrement per iteration (v_sub_u32 x, x, 1
    // clamp: a lane that left holds 0), the flag being x != 0, with
    // MK_JIT_SAT_BLOCK (4, 8, 16, 32) decrements per asm statement, so the
    // hazard recognizer's s_nop after an asm statement comes once per block
    // (r05h, C5 launch: block 4 120.6 us, 8 121.9, 16 121.6, 32 122.9, one
    // per statement 125.2-125.6).  Round 5 removed the superseded forms
    // (sub + min_u32 flags, one decrement per statement, usub.sat).
    uint32_t sat_block = 4;
    // ... and a countdown by any other step k (x > 0, x -= k; x < 0, x += k)
    // as one saturating decrement of its remaining-iteration count per
    // iteration (MK_JIT_SAT_COUNT=0: the bump and a med3 / shift flag).
    bool sat_count = true;
    // Two lanes per thread in the tile-sorted kernel when the network has no
    // stack slots: one sweep pass for two sorted chunks (MK_PAIR in
    // kMachineSortKernel; MK_JIT_PAIR=0: one lane per thread).
    bool pair = true;
    // The tile-sorted kernel's grid, for networks with stack slots in HBM
    // and batches of 2^18 inputs or more, measured over the first launches
    // (mk_exec.hip GridTune; MK_JIT_TUNE_GRID=0: the resident grid).
    bool tune_grid = true;
    // Heavy stream networks whose LDS slots allow fewer than four waves per
    // CU keep more stack entries in registers until they do (MK_JIT_TUNE_REGS,
    // mk_exec.hip tune_soft_regs).
    bool tune_regs = true;
    // Heavy stream networks whose slots do not fit lds_slot_bytes keep the
    // first lds_slot_bytes / 256 of them in LDS and the rest in HBM, when
    // that is at least this percentage of them (MK_JIT_LDS_SPLIT; 0: HBM only).
    uint32_t lds_split = 75;
    // Diagnostics: the tile-sorted machine kernel reports shader-clock cycles
    // per phase (sort, chunks, loop and other variants, results) and its
    // dispatch rounds in place of the launch's counters (MK_JIT_PROF=1;
    // tools/probe/c5_decomp.py).  The launch's statistics are then not counts.
    bool prof = false;

    // VGPRs per SIMD lane a module's waves share when a stack plan's module
    // is checked against its waves per SIMD (mk_exec.hip module_holds):
    // gfx950's 512.  MK_JIT_VGPR_FILE lowers it so that tests reach the
    // rejection path (the next plan, last the default) on purpose.
    uint32_t vgpr_file = 512;

    static JitLimits from_env();
    // The knobs that change generated code, as text (the module cache key
    // and the `knobs=` field of mk_net_plan).
    std::string key() const;
};

// The lane source for `p` in portable C++ (host g++ or HIP device).  Both
// shapes define
//   MK_FN int32_t mk_lane(int64_t in, uint32_t budget, int32_t *slots,
//                         uint64_t sstride, uint32_t *steps, uint32_t *status)
// (the machine shape builds it from mk_init/mk_run, driving MK_LOOP_NEED /
// MK_KEEP / MK_ALL; slot accesses go through MK_SLOT_ST / MK_SLOT_LD; the
// includer defines all five).  `slots` points at stack slot 0 of the lane,
// slot s at slots[s * sstride].  MK_FN is defined by the includer.
// Returns false (why) when over limits.
// max_steps: the stream shape's longest path in retired instructions (its
// kernel serves launches with a larger budget only); UINT64_MAX for machine.
// heavy: more than lim.heavy_ops micro-ops emitted (the stream shape then
// runs one lane per thread in 64-thread blocks instead of 4-lane tiles).
// The checked lane (mk_lane of the stream shape) is emitted only with
// `checked` (host tests); the GPU module does not compile it.
// pool: slots per wave of the machine shape's lane pool (0: pool-less kernel).
bool jit_lane_source(const SchedProgram &p, const JitLimits &lim, std::string &src, std::string &why,
                     JitShape *shape = nullptr, uint64_t *max_steps = nullptr, bool *heavy = nullptr,
                     bool checked = false, uint32_t *pool = nullptr);

// Whether the heavy stream kernel keeps the lane's `nslots` stack slots in
// LDS (the executor then allocates no HBM slots and launches one grid).
bool jit_slots_in_lds(uint32_t nslots, bool heavy, const JitLimits &lim);
// Slots of the lane the heavy stream kernel keeps in LDS: all (jit_slots_in_lds),
// the first ones with JitLimits::lds_split, or none.
uint32_t jit_lds_slot_count(uint32_t nslots, bool heavy, const JitLimits &lim);

// Full hiprtc translation unit: prelude, shared device code
// (mk_device_common.inc), the lane source and the kernel `mk_jit_exec` of
// the given shape.
// lim.policy (the machine shape's policy word) is compiled in.
std::string jit_module_source(const std::string &lane_src, JitShape shape, bool heavy, const JitLimits &lim,
                              uint32_t pool = 0);

// Lanes per thread per tile of the tile-sorted machine kernel (MK_TS_R):
// JitLimits::ts_rounds_slots for lanes with stack slots, else ts_rounds, or
// by the lane's stack slots when that is 0.  jit_compile compiles the module
// with it (the prelude's MK_TS_R), launch_jit_locked sizes the grid by it.
inline uint32_t jit_sort_rounds(const JitLimits &lim, uint32_t nslots)
{
    if (nslots && lim.ts_rounds_slots) return lim.ts_rounds_slots;
    return lim.ts_rounds ? lim.ts_rounds : nslots ? 4u : 8u;
}

// Name of the generated kernel.
constexpr const char *kJitKernel = "mk_jit_exec";
constexpr int kJitBlock = 256;
constexpr int kJitStreamLanes = 4; // lanes per thread per tile (stream shape)
constexpr int kJitHeavyBlock = 64;
// Machines of kSweepMinVariants to kSweepMaxVariants reachable variants
// dispatch by sweeps first (JitLimits::sweep).
constexpr size_t kSweepMinVariants = 16, kSweepMaxVariants = 128;
constexpr int kJitPoolBlock = 64;         // the pool kernel: one wave per block, its own pool
constexpr size_t kJitPoolBytes = 12288;   // LDS for one wave's lane pool (slots = bytes / lane state)
constexpr uint32_t kJitPoolMaxSlots = 256;
constexpr uint32_t kJitPoolMinSlots = 128;
constexpr size_t kJitPoolMaxVariants = 1024; // LDS histogram of parked lanes per superblock variant
// Heavy-kernel slot layout: up to this many slots per lane, wave-blocked
// ([wave][slot][64 lanes]: a wave's stacks are one contiguous block, read
// and written by buffer ops whose slot offset s * 256 is a scalar, which
// bounds the block to 2^31 bytes); above it, lane-major ([slot][lanes]).
// Measured on MI355X: C4 d64 (328 slots) 577 -> 539 us blocked; d256 (1,864
// slots) 1.51 -> 1.32 ms blocked, 1.23 ms with buffer ops; d1024 (8,008
// slots) with pipelined pops 2.97 ms blocked vs 3.18 ms lane-major (before
// the buffer ops, blocked held 116 VGPRs and lost: 4.14 vs 3.42 ms).
// MK_JIT_SLOT_LAYOUT=blocked|lane forces one.
constexpr uint32_t kJitWaveBlockedSlots = 1u << 22;

// Stateful sessions (row f2): the session schedule (compile_session_schedule)
// as a machine-shape lane plus the kernel kJitSessKernel, one thread per
// session, state in HBM; handed-off calls go to the interpreter.
constexpr const char *kJitSessKernel = "mk_sess_exec";
bool jit_session_source(const SchedProgram &p, const JitLimits &lim, std::string &src, std::string &why);
// Longest call of a session schedule in retired node-instructions
// (UINT64_MAX: unbounded, a call can loop); see tis_jit.cpp.
uint64_t jit_session_max_call_steps(const SchedProgram &p, const JitLimits &lim);
// The lane part alone (CPU tests compile it with g++).
bool jit_session_lane(const SchedProgram &p, const JitLimits &lim, std::string &src, std::string &why);

} // namespace mk
