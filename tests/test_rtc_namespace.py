"""Which compiler builds the native tier's modules (mk_exec.hip rtc_choice).

In a process that imported PyTorch first, the linked hiprtc symbols resolve
to PyTorch's bundled copy; the library then compiles with this ROCm's hiprtc
opened in a link-map namespace of its own (dlmopen), on one compile thread.
No GPU is needed: mk_net_plan compiles the module.  Each case runs in a
subprocess so that the process's import order is the one under test."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_PROG = r"""
import os, sys
sys.path[:0] = [{root!r}, os.path.join({root!r}, "tests")]
if {torch!r}:
    import torch  # noqa: F401  (PyTorch's bundled hiprtc resolves first)
import misaka_net_amd as mk
from tisgen import loop_cases, random_network
nets = [n for _, n, _, _ in loop_cases(n=16)][:{nloop}] + [random_network(s) for s in range({nrand})]
seen = {{}}
for nodes in nets:
    p = mk.Network(nodes).plan()
    r = p.split("rtc=")[1].split()[0] if "rtc=" in p else p.split()[0]
    seen[r] = seen.get(r, 0) + 1
threads = len(os.listdir("/proc/self/task"))
print("RESULT", sorted(seen.items()), threads, flush=True)
"""


def _run(torch: bool, nloop: int, nrand: int, env=None):
    code = _PROG.format(root=ROOT, torch=torch, nloop=nloop, nrand=nrand)
    e = dict(os.environ)
    e.pop("MK_HIPRTC", None)
    e.update(env or {})
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600, env=e)
    assert r.returncode == 0, (r.returncode, r.stderr[-3000:])
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT")][-1]
    return line


def test_pytorch_process_compiles_in_namespace():
    # every module by this ROCm's compiler in process (no helper child)
    line = _run(True, 13, 24)
    assert "('ns', 37)" in line, line


def test_plain_process_uses_linked_hiprtc():
    # a C / cgo caller's situation: the linked hiprtc is this ROCm's
    line = _run(False, 4, 2)
    assert "('linked', 6)" in line, line


def test_namespace_and_standalone_modules_are_identical(tmp_path):
    # the namespace copy is this ROCm's compiler: its code object is
    # byte-identical to the standalone test compiler's (a process that never
    # loads PyTorch) for the same generated source
    import schedcheck as sc

    code = r"""
import os, sys
sys.path[:0] = [{root!r}]
import torch  # noqa: F401
import misaka_net_amd as mk
print(mk.Network(mk.networks.pipeline_network(256)).plan().split("rtc=")[1].split()[0])
"""
    dump = str(tmp_path / "ns.co")
    e = dict(os.environ, MK_HIPRTC="ns", MK_JIT_DUMP=dump)
    r = subprocess.run([sys.executable, "-c", code.format(root=ROOT)], capture_output=True, text=True,
                       timeout=600, env=e)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.split()[-1] == "ns"
    alone = str(tmp_path / "alone.co")
    t = subprocess.run([sc.rtc_tool(), dump + ".hip", alone], capture_output=True, text=True, timeout=600)
    assert t.returncode == 0, t.stdout[-2000:]
    with open(dump, "rb") as f, open(alone, "rb") as g:
        a, b = f.read(), g.read()
    assert a and a == b


@pytest.mark.parametrize("mode", ["helper", "/usr/bin/true"])
def test_helper_process_compiler_is_refused(mode):
    # the round-3 helper child process (posix_spawn from a compile thread of
    # a GPU-initialised process) no longer exists: asking for
    # it keeps the network off the native tier, with the reason in the plan
    code = r"""
import os, sys
sys.path[:0] = [{root!r}]
import misaka_net_amd as mk
print("RESULT", mk.Network(mk.networks.example_network()).plan())
"""
    e = dict(os.environ, MK_HIPRTC=mode)
    r = subprocess.run([sys.executable, "-c", code.format(root=ROOT)], capture_output=True, text=True, timeout=600,
                       env=e)
    assert r.returncode == 0, r.stderr[-2000:]
    plan = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT")][-1]
    assert "tier=compiled" in plan and "MK_HIPRTC" in plan and "rtc=" not in plan, plan


@pytest.mark.parametrize("torch_first", [True])
def test_namespace_compiles_keep_one_thread(torch_first):
    # the compile thread is created once; compiles on short-lived threads
    # would call the namespace's libc from threads it never initialised
    a = _run(torch_first, 2, 0).split()[-1]
    b = _run(torch_first, 13, 10).split()[-1]
    assert a == b, (a, b)


def test_namespace_ctype_needs_the_opening_thread(tmp_path):
    # the hazard the single compile thread avoids, in 20 lines of C: a
    # dlmopen'd library's ctype calls from a thread other than the one that
    # opened the namespace read uninitialised thread-local tables
    lib_c = tmp_path / "ct.c"
    lib_c.write_text("#include <ctype.h>\nint ns_isalpha(int c) { return isalpha(c) != 0; }\n")
    main_c = tmp_path / "m.c"
    main_c.write_text(r"""
#define _GNU_SOURCE
#include <dlfcn.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
static int (*f)(int);
static void *t(void *a) { (void)a; printf("%d\n", f('a')); fflush(stdout); return 0; }
int main(int argc, char **argv) {
  void *h = dlmopen(LM_ID_NEWLM, argv[1], RTLD_NOW);
  if (!h) return 2;
  f = (int (*)(int))dlsym(h, "ns_isalpha");
  printf("%d\n", f('a')); fflush(stdout);
  if (argc > 2) { pthread_t th; pthread_create(&th, 0, t, 0); pthread_join(th, 0); }
  return 0;
}
""")
    so, exe = tmp_path / "libct.so", tmp_path / "m"
    subprocess.check_call(["gcc", "-shared", "-fPIC", str(lib_c), "-o", str(so)])
    subprocess.check_call(["gcc", str(main_c), "-o", str(exe), "-ldl", "-lpthread"])
    same = subprocess.run([str(exe), str(so)], capture_output=True, text=True, timeout=30)
    assert same.returncode == 0 and same.stdout.split() == ["1"]
    other = subprocess.run([str(exe), str(so), "other"], capture_output=True, text=True, timeout=30)
    assert other.returncode == -11, (other.returncode, other.stdout)


def test_namespace_survives_setenv_between_compiles():
    # setenv reallocates the environment array the namespace's libc was
    # opened with; every compile hands the namespace a fresh private copy
    code = r"""
import os, sys
sys.path[:0] = [{root!r}]
import torch  # noqa: F401
import misaka_net_amd as mk
for i in range(4):
    os.environ[f"MK_PRE_{{i}}"] = "x"
a = mk.Network(mk.networks.example_network()).plan().split("rtc=")[1].split()[0]
for i in range(200):
    os.environ[f"MK_POST_{{i}}"] = "y" * 50
b = mk.Network(mk.networks.countdown_network()).plan().split("rtc=")[1].split()[0]
print("RESULT", a, b)
"""
    e = dict(os.environ)
    e.pop("MK_HIPRTC", None)
    r = subprocess.run([sys.executable, "-c", code.format(root=ROOT)], capture_output=True, text=True, timeout=600,
                       env=e)
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
    assert r.stdout.split()[-2:] == ["ns", "ns"], r.stdout


@pytest.mark.parametrize("mode", ["linked", "ns"])
def test_compile_past_its_bound_does_not_hold_the_next(mode):
    """A compile that outlives its bound (MK_JIT_COMPILE_S) keeps its LLVM
    busy until it ends; the next network's compile takes another namespace
    worker (NsPool) instead of waiting out its own bound behind it and falling
    back to tier 2.  AMD_COMGR_CACHE=0: the slow module really compiles."""
    code = r"""
import os, sys, time
sys.path[:0] = [{root!r}]
import misaka_net_amd as mk
big = mk.Network(mk.networks.pipeline_network(256)).plan()
t = time.time()
small = mk.Network(mk.networks.example_network()).plan()
print("RESULT", big.split()[0], small.split()[0], round(time.time() - t, 2), flush=True)
"""
    # bound 2.5 s: D = 256 compiles in ~4.4 s (round 6), past it; the small
    # network alone in ~0.9 s, whose margin under a 1 s bound was too thin
    # with the big compile running beside it
    e = dict(os.environ, MK_HIPRTC=mode, MK_JIT_COMPILE_S="2.5", AMD_COMGR_CACHE="0", MK_JIT_TUNE_REGS="0")
    r = subprocess.run([sys.executable, "-c", code.format(root=ROOT)], capture_output=True, text=True, timeout=600,
                       env=e)
    assert r.returncode == 0, r.stderr[-3000:]
    _, big, small, secs = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT")][-1].split()
    assert big == "tier=compiled", big  # D = 256 takes hiprtc ~4.4 s: past the 2.5 s bound
    assert small == "tier=native" and float(secs) < 3.5, (small, secs)
