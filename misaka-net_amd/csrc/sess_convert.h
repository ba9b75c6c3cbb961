// sess_convert.h -- a stateful session handed off by the native tier
// (U_HANDOFF at the entry of a superblock) in the bytecode interpreter's
// terms: instruction pointers, ACC / BAK, ports, pending sends, stacks, the
// master's inChan / outChan and the open call (its input, whether it is
// deposited, where the round stands).  One restatement for the GPU import
// kernel (mk_exec.hip sess_import_one) and the host model's CPU tests
// (sched_check.cpp): the map comes from the schedule compiler
// (tis_sched.h SessMapHdr / SessSrcDev), the data from the lane's
// registers and stack slots.
//
//   Out: acc(n, v) bak(n, v) ip(n, v) pendv(n, v) port(q, v) pfull(x)
//        bits(pend, hung) chans(in_full, out_full, in_val, out_val)
//        depth(s, d) entry(s, d, v) call(deposited, pin, pos, changed)
#pragma once

#ifndef MK_HD
#define MK_HD
#endif

namespace mk {

template <class Reg, class Slot>
MK_HD inline int64_t sess_value(const SessSrcDev &x, const Reg &reg, const Slot &slot)
{
    return x.kind == 1u ? x.c : x.kind == 2u ? reg(x.r) : x.kind == 3u ? (int64_t)slot(x.r) : 0;
}

template <class Reg, class Slot, class Out>
MK_HD inline void sess_convert(int N, int S, const SessMapHdr &h, const SessSrcDev *rec, const int64_t *dyn_base,
                               const Reg &reg, const Slot &slot, Out &o)
{
    const SessSrcDev *ip = rec, *loc = rec + N;
    auto v64 = [&](int X) { return sess_value(loc[X], reg, slot); };
    auto v32 = [&](int X) { return (int32_t)(uint32_t)(uint64_t)v64(X); };
    for (int n = 0; n < N; n++) {
        o.ip(n, (int32_t)ip[n].c);
        o.acc(n, v64(n));
        o.bak(n, v64(N + n));
        o.pendv(n, v32(6 * N + n));
    }
    for (int q = 0; q < 4 * N; q++) o.port(q, ((h.pfull >> q) & 1ull) ? v32(2 * N + q) : 0);
    o.pfull(h.pfull);
    o.bits(h.pend, h.hung);
    const bool in_full = h.flags & 1u, out_full = h.flags & 2u, dep = h.flags & 4u;
    o.chans(in_full, out_full, in_full ? v32(7 * N) : 0, out_full ? v32(7 * N + 1) : 0);
    const SessSrcDev *sr = loc + 7 * N + 2 + S + 1; // after CIN
    for (int s = 0; s < S; s++) {
        const uint32_t k = (uint32_t)sr->c;
        ++sr;
        if (dyn_base[s] >= 0) { // a dynamic stack: DEP entries in slots base + j
            const uint32_t d = (uint32_t)v64(7 * N + 2 + s);
            o.depth(s, d);
            for (uint32_t j = 0; j < d; j++) o.entry(s, j, (int32_t)slot((uint32_t)dyn_base[s] + j));
        } else {
            o.depth(s, k);
            for (uint32_t j = 0; j < k; j++) o.entry(s, j, (int32_t)sess_value(sr[j], reg, slot));
        }
        sr += k;
    }
    o.call(dep, dep ? 0 : v32(7 * N + 2 + S), (int)(h.flags >> 8) & 0xff, (h.flags & 8u) != 0);
}

} // namespace mk
