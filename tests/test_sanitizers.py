"""ASAN + UBSAN run of the host code (SURVEY.md §5 "Race detection / sanitizers"; the reference's opt-in analysis is
cmake/static_analysis.cmake:2-22): tools/sanitize builds the CPU oracle, the scene synthesiser and the host half of
the C ABI (globals / ECS feed, render graph, PNG / EXR writers) with -fsanitize=address,undefined (host code only)
and runs a driver over all of them: every oracle pass on even and odd extents, the graph's construction, caller
passes, ring edges and error paths. Any sanitizer report aborts the driver (-fno-sanitize-recover). CPU only."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "tools", "sanitize")


def test_host_code_under_asan_ubsan(tmp_path):
    b = subprocess.run(["make", "-s", "-C", SAN, "-j8"], capture_output=True, text=True, timeout=600)
    assert b.returncode == 0, b.stdout + b.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1", SAN_TMP=str(tmp_path))
    p = subprocess.run([os.path.join(SAN, "build", "san_host")], capture_output=True, text=True, timeout=600, env=env)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-4000:]
    assert "san_host: ok (0 failed checks)" in p.stdout
    assert "runtime error" not in out and "AddressSanitizer" not in out and "LeakSanitizer" not in out
    assert (tmp_path / "san_host.png").stat().st_size > 0 and (tmp_path / "san_host.exr").stat().st_size > 0
