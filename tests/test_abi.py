"""The C-ABI library loads without a GPU and exports every entry point that
include/mk.h declares; the product path refuses to run without its library."""
import ctypes
import os
import re

import pytest

import misaka_net_amd as mk

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    text = open(os.path.join(ROOT, "include", "mk.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mk_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_expected_api():
    names = declared_functions()
    for required in ["mk_net_load", "mk_net_free", "mk_compute_batch", "mk_compute_device"]:
        assert required in names


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(mk._native.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    assert set(declared_functions()) <= set(mk._native.SIGNATURES)


def test_library_is_gfx950_code_object():
    data = open(mk._native.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_version():
    assert b"gfx950" in mk._native.lib().mk_version()


def test_compute_without_gpu_fails_loudly():
    import torch

    if torch.cuda.is_available():
        return
    net = mk.Network(mk.networks.example_network())
    try:
        net.compute_batch([1, 2, 3])
    except mk._native.MkError as e:
        assert e.code == mk._native.MK_EDEVICE
    else:
        raise AssertionError("compute_batch must not succeed without a GPU")


def test_go_adapter_binds_only_declared_symbols():
    # integration/go/mk/mk.go (row f3, source only: no Go toolchain here) calls
    # the C ABI through cgo; every C.mk_* it names must exist in include/mk.h
    src = open(os.path.join(ROOT, "integration", "go", "mk", "mk.go")).read()
    used = set(re.findall(r"\bC\.(mk_[a-z_0-9]+)\b", src))
    types = {"mk_net", "mk_session", "mk_opts", "mk_node_desc", "mk_remote_req", "mk_trace_entry"}
    assert used - types <= set(declared_functions()), used - types - set(declared_functions())
    assert {"mk_net_load", "mk_compute_batch", "mk_session_create", "mk_session_compute", "mk_tokenize"} <= used


def test_go_master_adapter_routes_and_locking():
    # integration/go/gpumaster.go.txt (row f3, source only): every route of
    # master.go:90-224 plus /compute_batch; isRunning only under g.mu (the
    # reference reads and writes it unsynchronised, master.go:93,200)
    src = open(os.path.join(ROOT, "integration", "go", "gpumaster.go.txt")).read()
    routes = re.findall(r'post\("(/[a-z_]+)"', src)
    assert sorted(routes) == sorted(["/run", "/pause", "/reset", "/load", "/compute", "/compute_batch"]), routes
    for text in ("error loading program on node %s: %s", "node %s not valid on this network",
                 "network is not running", "cannot parse form", "cannot parse value", "method GET not allowed",
                 "error resetting network: %s"):
        assert text in src, text
    # every isRunning access sits in a region holding g.mu: within a function,
    # after a g.mu.Lock() with no g.mu.Unlock() since, or in a function whose
    # comment says the caller holds it
    funcs = re.split(r"\n(?=func |\tpost\()", src)
    for f in funcs:
        for m in re.finditer(r"g\.isRunning", f):
            before = f[:m.start()].replace("defer g.mu.Unlock()", "")
            held = before.rfind("g.mu.Lock()") > before.rfind("g.mu.Unlock()") or "g.mu held" in f
            assert held, f[:200]
    # /load resets under the lock before it reloads: both in the one handler
    load = src[src.index('post("/load"'):src.index('post("/compute"')]
    assert load.index("g.mu.Lock()") < load.index("g.sess.Reset()") < load.index("g.build()")


def _build_c_client(tmp_path):
    """integration/c/mk_client.c compiled by gcc against include/mk.h and the
    in-tree library: a compiled (non-Python) client of the boundary, making
    the cgo backend's calls."""
    import subprocess

    lib = os.path.dirname(mk._native.LIB_PATH)
    exe = str(tmp_path / "mk_client")
    subprocess.check_call(["gcc", "-std=c99", "-O2", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "integration", "c", "mk_client.c"), "-L", lib, "-lmisaka_amd",
                           f"-Wl,-rpath,{lib}", "-o", exe])
    return exe


def test_c_client_load_errors_and_no_gpu(tmp_path):
    import subprocess

    exe = _build_c_client(tmp_path)
    r = subprocess.run([exe, "-p", "MOV 1,ACC", "5"], capture_output=True, text=True)
    assert r.returncode == 2 and r.stdout == "load -2: node misaka1: line 0, 'MOV 1,ACC' not a valid instruction\n"
    r = subprocess.run([exe, "-p", "JMP NOWHERE", "5"], capture_output=True, text=True)
    assert r.returncode == 2 and "line 0, label 'NOWHERE' was not declared" in r.stdout
    import torch

    if not torch.cuda.is_available():  # no GPU here: the compute call fails loudly (MK_EDEVICE)
        r = subprocess.run([exe, "5"], capture_output=True, text=True)
        assert r.returncode == 3 and r.stdout == "compute -4\n"


def _build_c_bench(tmp_path):
    """integration/c/mk_bench.c: the batched path timed through the ABI alone
    (no PyTorch in the process), HIP runtime for buffers and events."""
    import subprocess

    lib = os.path.dirname(mk._native.LIB_PATH)
    exe = str(tmp_path / "mk_bench")
    subprocess.check_call(["gcc", "-std=c99", "-O2", "-Wall", "-Wextra", "-Werror", "-D__HIP_PLATFORM_AMD__",
                           "-I", os.path.join(ROOT, "include"), "-I", "/opt/rocm/include",
                           os.path.join(ROOT, "integration", "c", "mk_bench.c"), "-L", lib, "-lmisaka_amd",
                           "-L", "/opt/rocm/lib", "-lamdhip64", f"-Wl,-rpath,{lib}", "-Wl,-rpath,/opt/rocm/lib",
                           "-o", exe])
    return exe


@pytest.mark.parametrize("depth", [64, 256, 1024, "c5"])
def test_c_bench_networks_match_bench_py(tmp_path, depth):
    # the C timing client runs bench.py's networks: same program text
    import subprocess

    exe = _build_c_bench(tmp_path)
    wl = depth if depth == "c5" else f"c4:{depth}"
    r = subprocess.run([exe, wl, "print"], capture_output=True, text=True, check=True)
    got = {}
    for block in r.stdout.split("== ")[1:]:
        head, _, text = block.partition("\n")
        name, kind = head.split()
        got[name] = (int(kind), text)
    want = {n.name: ({"program": 0, "stack": 1}[n.kind], n.program if n.kind == "program" else "")
            for n in (mk.networks.countdown_network() if depth == "c5" else mk.networks.pipeline_network(depth))}
    assert got == want


@pytest.mark.gpu
@pytest.mark.parametrize("wl", ["c2", "c4:64", "c5"])
def test_c_bench_on_gpu(gpu, tmp_path, wl):
    import json
    import subprocess

    exe = _build_c_bench(tmp_path)
    r = subprocess.run([exe, wl, "3", "1"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["plan"].startswith("tier=native") and "rtc=linked" in rec["plan"], rec["plan"]
    assert rec["node_instr_per_s"] > 0 and rec["results_per_launch"] == rec["lanes"]


@pytest.mark.gpu
def test_c_client_compute_on_gpu(gpu, tmp_path):
    import subprocess

    exe = _build_c_client(tmp_path)
    vals = ["5", "0", "2147483646", "2147483647", "-2147483648", "4294967301"]
    r = subprocess.run([exe] + vals, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    got = [line.split() for line in r.stdout.splitlines()]
    assert [g[1] for g in got] == ["7", "2", "-2147483648", "-2147483647", "-2147483646", "7"]
    assert all(g[2] == "0x11" and g[3] == "12" for g in got)
