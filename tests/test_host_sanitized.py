"""Host-side memory safety of the untrusted-input paths (ASan /
UBSan on the C++ CPU path): the FriProof wire decoder (csrc/wire.hip) and the
FRI / PCS / batched verifiers (csrc/verify.cpp) built with
-fsanitize=address,undefined and driven by tests/fuzz/fuzz_verify.cpp over
thousands of mutations of a valid encoded proof (the oracle's proof of a
2^7-element RS codeword), plus inconsistent verifier headers.  CPU only."""
import os
import shutil
import subprocess

import pytest

from oracle import field as F
from oracle import fri as OF
from oracle import transcript as OT
from oracle import wire as OW

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "multilinear_amd", "csrc")


@pytest.fixture(scope="module")
def fuzzer(tmp_path_factory):
    cxx = shutil.which("g++")
    if not cxx:
        pytest.skip("g++ not available")
    d = tmp_path_factory.mktemp("fuzz")
    exe = str(d / "fuzz_verify")
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-o", exe, os.path.join(ROOT, "tests", "fuzz", "fuzz_verify.cpp"),
           os.path.join(CSRC, "verify.cpp"), "-x", "c++", os.path.join(CSRC, "wire.hip")]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    return exe, d


def _seed_proof(log_n):
    vals = [F.from_i64(7 * i + 3) for i in range(1 << log_n)]
    gp = F.pow_2_generator_powers(log_n + 1)
    code = OF.reed_solomon(vals, gp[1])
    return OW.encode_fri_proof(OF.FriProof.prove(code, gp, OT.Transcript()))


@pytest.mark.parametrize("log_n", [1, 6])
def test_fuzz_decode_and_verify_under_asan_ubsan(fuzzer, log_n):
    exe, d = fuzzer
    seed = d / ("seed_%d.bin" % log_n)
    seed.write_bytes(_seed_proof(log_n))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe, str(seed), "20000"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "fuzz ok" in r.stdout
