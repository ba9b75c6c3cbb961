/*
 * mk_bench.c -- what a cgo / C drop-in gets: times the batched /compute path
 * through include/mk.h alone, in a process that never loads PyTorch (so the
 * native tier's module comes from this ROCm's hiprtc, linked by the
 * library, exactly as in a Go binary that links libmisaka_amd.so).
 *
 * Workloads (bench.py's): "c2" = the docker-compose example network
 * (docker-compose.yml:35-40,54-59), 16,777,216 lanes; "c4:D" = the 8-node
 * pipeline with stack depth D (networks.py pipeline_program) at bench.py's
 * lane counts (D=64: 1M, D=256: 512K, D=1024: 256K).  Inputs are generated on
 * the device (mk_generate_inputs_device, the MK_GEN_FULL generator of
 * bench.py) and stay resident; each step is one mk_compute_device launch with
 * MK_FLAG_DEFER_STATS, timed with HIP events on the launch stream after
 * warm-up launches.  Prints one JSON line:
 *   {"client": "c", "workload": ..., "lanes": N, "steps": K, "ms_per_step": T,
 *    "node_instr_per_s": V, "plan": "..."}
 *
 * "c5" = the countdown network (networks.py countdown_network), 4,194,304
 * lanes of inputs masked to 0..1023 (bench.py's MK_GEN_MASKED generator).
 *   mk_bench [c2 | c4:D | c5] [steps] [warmup]
 * Exit codes: 0 ok, 2 load failed, 3 device / compute failed.
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mk.h"

static const char *MISAKA1 = "IN ACC\nADD 1\nMOV ACC, misaka2:R0\nMOV R0, ACC\nOUT ACC\n";
static const char *MISAKA2 = "MOV R0, ACC\nADD 1\nPUSH ACC, misaka3\nPOP misaka3, ACC\nMOV ACC, misaka1:R0\n";
/* networks.py countdown_network (C5) */
static const char *COUNT = "IN ACC\nSAV\nL: SUB 1\nJGZ L\nSWP\nMOV ACC, digits:R0\n";
static const char *DIGITS = "MOV R0, ACC\nJEZ Z\nJLZ Z\nL: SUB 3\nJGZ L\nADD 3\nJRO ACC\nADD 100\nADD 10\nADD 1\n"
                            "OUT ACC\nJMP E\nZ: OUT -1\nE: NOP\n";

/* networks.py pipeline_program(k, nodes, depth), line for line */
static char *pipeline_program(int k, int nodes, int depth)
{
    char *s = malloc(1024);
    int n = 0;
    if (k == 0) n += sprintf(s + n, "IN ACC\n");
    else n += sprintf(s + n, "MOV R0, ACC\n");
    n += sprintf(s + n, "SAV\nMOV %d, ACC\nPL: SWP\nADD 1\nPUSH ACC, s%d\nSWP\nSUB 1\nJGZ PL\n", depth, k);
    n += sprintf(s + n, "MOV 0, ACC\nSAV\nMOV %d, ACC\nMOV ACC, p%d:R1\n", depth, k);
    n += sprintf(s + n, "QL: POP s%d, ACC\nMOV ACC, p%d:R2\nSWP\nMOV ACC, p%d:R3\nADD ACC\nADD R3\nADD R2\nSAV\n", k, k,
                 k);
    n += sprintf(s + n, "MOV R1, ACC\nSUB 1\nMOV ACC, p%d:R1\nJGZ QL\nMOV R1, NIL\nSWP\n", k);
    if (k == nodes - 1) sprintf(s + n, "OUT ACC\n");
    else sprintf(s + n, "MOV ACC, p%d:R0\n", k + 1);
    return s;
}

#define CHECK_HIP(x)                                                             \
    do {                                                                         \
        if ((x) != hipSuccess) {                                                 \
            printf("{\"error\": \"%s failed at line %d\"}\n", #x, __LINE__);     \
            return 3;                                                            \
        }                                                                        \
    } while (0)

int main(int argc, char **argv)
{
    const char *wl = argc > 1 ? argv[1] : "c2";
    const int steps = argc > 2 ? atoi(argv[2]) : 20;
    const int warmup = argc > 3 ? atoi(argv[3]) : 3;
    mk_node_desc nodes[17];
    char names[16][8];
    char *progs[8] = {0};
    int nn = 0;
    size_t lanes = 0;
    uint32_t gen_kind = MK_GEN_FULL, gen_mask = 0; /* bench.py WORKLOADS' generator */
    if (!strcmp(wl, "c2")) {
        nodes[0] = (mk_node_desc){"misaka1", MK_NODE_PROGRAM, MISAKA1};
        nodes[1] = (mk_node_desc){"misaka2", MK_NODE_PROGRAM, MISAKA2};
        nodes[2] = (mk_node_desc){"misaka3", MK_NODE_STACK, NULL};
        nn = 3;
        lanes = (size_t)1 << 24;
    } else if (!strcmp(wl, "c5")) {
        nodes[0] = (mk_node_desc){"count", MK_NODE_PROGRAM, COUNT};
        nodes[1] = (mk_node_desc){"digits", MK_NODE_PROGRAM, DIGITS};
        nn = 2;
        lanes = (size_t)1 << 22;
        gen_kind = MK_GEN_MASKED, gen_mask = 1023;
    } else if (!strncmp(wl, "c4:", 3)) {
        const int depth = atoi(wl + 3);
        for (int k = 0; k < 8; ++k) {
            progs[k] = pipeline_program(k, 8, depth);
            snprintf(names[k], sizeof names[k], "p%d", k);
            snprintf(names[8 + k], sizeof names[8 + k], "s%d", k);
            nodes[nn++] = (mk_node_desc){names[k], MK_NODE_PROGRAM, progs[k]};
        }
        for (int k = 0; k < 8; ++k) nodes[nn++] = (mk_node_desc){names[8 + k], MK_NODE_STACK, NULL};
        lanes = depth <= 64 ? (size_t)1 << 20 : depth <= 256 ? (size_t)1 << 19 : (size_t)1 << 18;
    } else {
        printf("{\"error\": \"unknown workload %s\"}\n", wl);
        return 2;
    }
    if (argc > 2 && !strcmp(argv[2], "print")) { /* the network's text, no GPU (tests/test_abi.py) */
        for (int k = 0; k < nn; ++k) printf("== %s %d\n%s", nodes[k].name, nodes[k].kind, nodes[k].program ? nodes[k].program : "");
        return 0;
    }
    char err[512];
    mk_net *net = NULL;
    if (mk_net_load(nodes, nn, &net, err, sizeof err) != MK_OK) {
        printf("{\"error\": \"load: %s\"}\n", err);
        return 2;
    }
    mk_opts opts;
    memset(&opts, 0, sizeof opts);
    opts.flags = MK_FLAG_DEFER_STATS;
    int32_t *d_in = NULL, *d_out = NULL;
    uint8_t *d_st = NULL;
    uint64_t *d_stats = NULL;
    hipStream_t s;
    CHECK_HIP(hipSetDevice(0));
    CHECK_HIP(hipStreamCreate(&s));
    CHECK_HIP(hipMalloc((void **)&d_in, lanes * 4));
    CHECK_HIP(hipMalloc((void **)&d_out, lanes * 4));
    CHECK_HIP(hipMalloc((void **)&d_st, lanes));
    CHECK_HIP(hipMalloc((void **)&d_stats, 8 * sizeof(uint64_t)));
    CHECK_HIP(hipMemset(d_stats, 0, 8 * sizeof(uint64_t)));
    if (mk_generate_inputs_device(0, 0x4D49534B41ull, gen_kind, gen_mask, 0, lanes, d_in, s) != MK_OK) return 3;
    mk_input in;
    memset(&in, 0, sizeof in);
    in.kind = MK_IN_I32;
    in.data = d_in;
    if (mk_net_prepare(net, &opts, 0) != MK_OK) {
        printf("{\"error\": \"prepare\"}\n");
        return 3;
    }
    for (int i = 0; i < warmup; ++i)
        if (mk_compute_device(net, 0, &in, lanes, d_out, d_st, NULL, NULL, &opts, s) != MK_OK) return 3;
    if (mk_stats_fold(net, 0, d_stats, s) != MK_OK) return 3;
    CHECK_HIP(hipStreamSynchronize(s));
    CHECK_HIP(hipMemset(d_stats, 0, 8 * sizeof(uint64_t)));
    hipEvent_t e0, e1;
    CHECK_HIP(hipEventCreate(&e0));
    CHECK_HIP(hipEventCreate(&e1));
    CHECK_HIP(hipEventRecord(e0, s));
    for (int i = 0; i < steps; ++i)
        if (mk_compute_device(net, 0, &in, lanes, d_out, d_st, NULL, NULL, &opts, s) != MK_OK) return 3;
    CHECK_HIP(hipEventRecord(e1, s));
    if (mk_stats_fold(net, 0, d_stats, s) != MK_OK) return 3;
    CHECK_HIP(hipStreamSynchronize(s));
    float ms = 0.f;
    CHECK_HIP(hipEventElapsedTime(&ms, e0, e1));
    uint64_t stats[8];
    CHECK_HIP(hipMemcpy(stats, d_stats, sizeof stats, hipMemcpyDeviceToHost));
    char plan[1024];
    if (mk_net_plan(net, &opts, plan, sizeof plan) != MK_OK) plan[0] = 0;
    for (char *c = plan; *c; ++c)
        if (*c == '"') *c = '\'';
    printf("{\"client\": \"c\", \"workload\": \"%s\", \"lanes\": %zu, \"steps\": %d, \"ms_per_step\": %.6f, "
           "\"node_instr_per_s\": %.6e, \"results_per_launch\": %.1f, \"plan\": \"%s\"}\n",
           wl, lanes, steps, ms / steps, (double)stats[0] / (ms * 1e-3), (double)stats[1] / steps, plan);
    hipFree(d_in);
    hipFree(d_out);
    hipFree(d_st);
    hipFree(d_stats);
    mk_net_free(net);
    for (int k = 0; k < 8; ++k) free(progs[k]);
    return 0;
}
