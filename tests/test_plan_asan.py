"""Host-side sanitizer run of the plan builders (CPU sanitizer build): every source compiled
with AddressSanitizer + UndefinedBehaviorSanitizer on the host side (`make asan`), driving
tools/plan_check.cpp over 676 cnn_small / cnn_deep configurations (B 1..32768, T 16..256, widths,
residual / plain, fp32 / bf16): each plan builds, reports its counts and gradient stages, and every named
cnn_small region lies inside the workspace behind the 256-byte guard.  No GPU is touched."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tools", "plan_check_asan")


def test_plan_builders_clean_under_asan_ubsan():
    # always through make (incremental): a sanitizer binary older than the plan builders would test old code
    r = subprocess.run(["make", "-j8", "asan"], cwd=ROOT, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "0 failures" in r.stdout and "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
