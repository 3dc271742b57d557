"""ASan+UBSan and TSan runs of the multi-threaded canonical reader
(das_amd/csrc/canonical.cpp, the host C++ in front of the device hashing).

`make -C das_amd/csrc asan tsan` builds the reader with plain g++ (no HIP
headers: it includes status.h only) together with tests/native/canonical_check.cpp,
which parses every input at 1-16 threads and three chunk sizes and requires
identical arrays; the sanitizer runtimes are linked into the executable, so no
preload is involved.  Inputs: the reference's canonical toy KB, seeded random
canonical texts (nesting, multi-word names, whitespace runs, CR/LF), a
FlyBase-shaped dump, and the reader's syntax-error cases (must be rejected).
CPU only."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from test_canonical_native import _random_canonical

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "das_amd", "csrc")
DATA = os.path.join(HERE, "golden", "data")

BAD = [
    '(: Concept Type)\n(Inheritance "Concept a" "Concept b")\n',
    '(: Concept Type)\n(: "a" Concept)\n(Inheritance "Concept a")\n(: "b" Concept)\n',
    '(: Concept Type)\n(: "a" Concept)\n(Inheritance "Concept a"\n',
    '(: Concept Type)\n(: "a" Concept)\n(Inheritance "Concept a)\n',
    '(: Concept Type Extra)\n(: "a" Concept)\n',
]


@pytest.fixture(scope="module")
def inputs(tmp_path_factory):
    from das_amd import synthetic
    d = tmp_path_factory.mktemp("canon")
    paths = []
    shutil.copy(os.path.join(DATA, "canonical_toy-example-mining.metta"), d / "toy.metta")
    paths.append(str(d / "toy.metta"))
    for seed, sep in ((1, "\n"), (2, "\r\n"), (3, "\r")):
        rng = np.random.default_rng(seed)
        p = d / f"random{seed}.metta"
        p.write_bytes((sep.join(_random_canonical(rng, n_lines=600, ws=True)) + sep).encode())
        paths.append(str(p))
    p = d / "flybase.metta"
    p.write_text(synthetic.to_canonical(synthetic.flybase_kb(300, 6, 400, n_loc=20, n_do=10)))
    paths.append(str(p))
    for i, t in enumerate(BAD):
        p = d / f"bad_{i}.metta"
        p.write_text(t)
        paths.append(str(p))
    return paths


@pytest.mark.parametrize("target", ["asan", "tsan"])
def test_canonical_reader_under_sanitizer(target, inputs):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    subprocess.run(["make", "-s", "-C", CSRC, target], check=True, timeout=600)
    exe = os.path.join(CSRC, "build", f"canonical_{target}")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=23",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=24",
               TSAN_OPTIONS="halt_on_error=1:exitcode=25")
    r = subprocess.run([exe] + inputs, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "OK" in r.stdout.splitlines()[-1]
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
