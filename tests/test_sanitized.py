"""The host code that takes untrusted program text -- the parser
(csrc/tis_front.cpp, tokenizer.go:11-106), the lowering and schedule
compiler (tis_sched.cpp, program.go:178-193), the session compiler and the
native-tier code generator (tis_jit.cpp) -- built with AddressSanitizer and
UndefinedBehaviorSanitizer (__graft_entry__.build_check(sanitize=True)) and
driven by the CPU tests of those components in a child pytest that loads
that build (MK_CHECK_LIB) with the ASan runtime preloaded.  Any report ends
the child (halt_on_error, -fno-sanitize-recover=undefined).

The default selection runs in about a minute: every front-end golden vector,
the schedule compiler on C2/C3/C5 and random networks, sessions, and the code
generator on random networks (the C4 pipelines take minutes under ASan).  MK_SAN_FULL=1 runs the four test files whole
(profiles/r06_sanitized_full.log holds such a run).  Host code only: GPU
code is never sanitized here."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

QUICK = [
    "tests/test_tokenizer_golden.py::test_check_library_front_end_matches_reference_regexes",
    "tests/test_sched_compiler.py::test_configs[c2_example]",
    "tests/test_sched_compiler.py::test_configs[c3_sample]",
    "tests/test_sched_compiler.py::test_configs[c5_countdown]",
    "tests/test_sched_compiler.py::test_budget_boundaries",
    "tests/test_sched_compiler.py::test_random_networks",
    "tests/test_sched_compiler.py::test_wide_immediates_on_symbolic_acc",
    "tests/test_sched_compiler.py::test_slot_sharing_is_safe",
    "tests/test_session_compiler.py::test_example_network_sessions",
    "tests/test_session_compiler.py::test_config_networks",
    "tests/test_session_compiler.py::test_long_call_hands_off_mid_loop",
    "tests/test_session_compiler.py::test_session_call_bound_covers_every_call",
    "tests/test_session_compiler.py::test_generated_session_lane",
    "tests/test_jit_codegen.py::test_random_networks[0-False]",
    "tests/test_jit_codegen.py::test_random_networks[1-True]",
    "tests/test_jit_codegen.py::test_wide_immediates_and_stop",
    "tests/test_jit_codegen.py::test_shapes",
]
FULL = ["tests/test_tokenizer_golden.py", "tests/test_sched_compiler.py", "tests/test_session_compiler.py",
        "tests/test_jit_codegen.py"]


def _asan_runtime():
    r = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True)
    p = r.stdout.strip()
    return p if r.returncode == 0 and os.path.isabs(p) and os.path.exists(p) else None


def test_compilers_under_asan_and_ubsan():
    import __graft_entry__ as g

    asan = _asan_runtime()
    if asan is None:
        pytest.skip("no ASan runtime for gcc in this image")
    lib = g.build_check(sanitize=True)
    env = dict(os.environ)
    env["LD_PRELOAD"] = " ".join([asan] + ([env["LD_PRELOAD"]] if env.get("LD_PRELOAD") else []))
    env["ASAN_OPTIONS"] = "detect_leaks=0:halt_on_error=1"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    env["MK_CHECK_LIB"] = lib
    sel = FULL if os.environ.get("MK_SAN_FULL") == "1" else QUICK
    r = subprocess.run([sys.executable, "-m", "pytest", *sel, "-x", "-q", "-p", "no:cacheprovider", "-m", "not gpu"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=3000)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out and "runtime error:" not in out, out[-6000:]
    assert r.returncode == 0, out[-4000:]
    assert " passed" in out
