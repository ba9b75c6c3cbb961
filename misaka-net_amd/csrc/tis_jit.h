// tis_jit.h -- tier 3: a network's compiled schedule (tis_sched.h) turned
// into straight-line code, one native kernel per (network, stack_cap,
// stop_on_output), compiled for gfx950 at run time by hiprtc.
//
// Superblock variants become labels, their micro-ops int64 expressions on
// local variables (VGPRs instead of the LDS register file of tier 2), exits
// become gotos (BR), a switch over the clamped operand (JRO), or the lane's
// result (END / ROUND_END).  Nothing is interpreted at run time: no fetch, no
// dispatch, no waterfall.  Divergent lanes of a wave are handled by the
// hardware's exec mask like any other branchy kernel.
#pragma once

#include <cstdint>
#include <string>

#include "tis_sched.h"

namespace mk {

struct JitLimits {
    uint32_t max_variants = 4096; // superblock variants (labels)
    size_t max_dops = 4096;       // micro-ops in the reachable code (hiprtc time grows
                                  // superlinearly: 14K straight-line ops take ~150 s)
};

// The lane function for `p` in portable C++ (host g++ or HIP device):
//   MK_FN int32_t mk_lane(int64_t in, uint32_t budget, int32_t *slots,
//                         uint64_t sstride, uint32_t *steps, uint32_t *status)
// `slots` points at stack slot 0 of the lane, slot s at slots[s * sstride].
// MK_FN is defined by the includer.  Returns false (why) when over limits.
bool jit_lane_source(const SchedProgram &p, const JitLimits &lim, std::string &src, std::string &why);

// Full hiprtc translation unit: prelude, shared device code
// (mk_device_common.inc), the lane function and the kernel `mk_jit_exec`.
std::string jit_module_source(const std::string &lane_src);

// Name of the generated kernel.
constexpr const char *kJitKernel = "mk_jit_exec";
constexpr int kJitBlock = 256;

} // namespace mk
