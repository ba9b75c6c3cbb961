/*
 * mk_client.c -- a compiled C client of include/mk.h: the call sequence the
 * cgo backend (integration/go/mk/mk.go, gpumaster.go.txt) makes, without Go.
 *
 * It loads the docker-compose example network (docker-compose.yml:35-40,
 * 54-59; NODE_INFO as cmd/app.go:31 reads it), answers /compute values given
 * on the command line in one mk_compute_batch call (master.go:197-224 for a
 * batch), and prints one line per value: "<value> <out> <status> <steps>".
 * A program argument replaces misaka1's text, so a rejected /load shows the
 * reference's error string (tokenizer.go:20,74,101).  Exit codes: 0 ok,
 * 2 load rejected, 3 compute failed (e.g. MK_EDEVICE without a GPU).
 *
 *   mk_client [-p PROGRAM_FOR_misaka1] [-s stack_cap] [-b budget] VALUE...
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mk.h"

static const char *MISAKA1 = "IN ACC\nADD 1\nMOV ACC, misaka2:R0\nMOV R0, ACC\nOUT ACC\n";
static const char *MISAKA2 = "MOV R0, ACC\nADD 1\nPUSH ACC, misaka3\nPOP misaka3, ACC\nMOV ACC, misaka1:R0\n";

int main(int argc, char **argv)
{
    const char *prog1 = MISAKA1;
    mk_opts opts;
    memset(&opts, 0, sizeof opts);
    int i = 1;
    for (; i + 1 < argc && argv[i][0] == '-' && argv[i][1] && !argv[i][2]; i += 2) {
        if (argv[i][1] == 'p') prog1 = argv[i + 1];
        else if (argv[i][1] == 's') opts.stack_cap = (uint32_t)strtoul(argv[i + 1], NULL, 10);
        else if (argv[i][1] == 'b') opts.budget = (uint32_t)strtoul(argv[i + 1], NULL, 10);
        else break;
    }
    const mk_node_desc nodes[] = {
        {"misaka1", MK_NODE_PROGRAM, prog1},
        {"misaka2", MK_NODE_PROGRAM, MISAKA2},
        {"misaka3", MK_NODE_STACK, NULL},
        {"last_order", MK_NODE_MASTER, NULL},
    };
    char err[512];
    mk_net *net = NULL;
    int rc = mk_net_load(nodes, 4, &net, err, sizeof err);
    if (rc != MK_OK) {
        printf("load %d: %s\n", rc, err);
        return 2;
    }
    const size_t n = (size_t)(argc - i);
    int64_t *in = calloc(n ? n : 1, sizeof *in);
    int32_t *out = calloc(n ? n : 1, sizeof *out);
    uint8_t *st = calloc(n ? n : 1, 1);
    uint32_t *steps = calloc(n ? n : 1, sizeof *steps);
    for (size_t k = 0; k < n; ++k) in[k] = strtoll(argv[i + k], NULL, 10);
    rc = mk_compute_batch(net, in, n, out, st, steps, &opts);
    if (rc != MK_OK) {
        printf("compute %d\n", rc);
        mk_net_free(net);
        return 3;
    }
    for (size_t k = 0; k < n; ++k)
        printf("%lld %d 0x%02x %u\n", (long long)in[k], out[k], st[k], steps[k]);
    free(in), free(out), free(st), free(steps);
    mk_net_free(net);
    return 0;
}
