/* orc_flat.h -- TEST INFRASTRUCTURE (see tis_oracle.c).  One stateful
 * session in the bytecode interpreter's terms, with an open /compute call:
 * what the native tier hands to the interpreter when a call's budget slice
 * ends inside a superblock (misaka-net_amd/csrc/sess_convert.h).  The
 * schedule compiler's host model (sched_check.cpp) exports it and the
 * oracle imports it (orc_session_import), so the hand-off is checked on
 * the CPU against the oracle's own run of the same calls. */
#ifndef ORC_FLAT_H
#define ORC_FLAT_H
#include <stdint.h>

#define ORC_FLAT_NODES 64

typedef struct {
    int64_t acc[ORC_FLAT_NODES], bak[ORC_FLAT_NODES];
    int32_t ip[ORC_FLAT_NODES], pendv[ORC_FLAT_NODES];
    int32_t port[4 * ORC_FLAT_NODES];
    uint64_t pfull;
    uint32_t pend, hung;
    int32_t in_full, out_full, in_val, out_val;
    uint32_t depth[ORC_FLAT_NODES];
    const int32_t *entries; /* [stack][stack_cap] */
    int32_t deposited, pin, pos, changed;
    uint32_t csteps;
} orc_flat;

#endif
