"""The host front-end on the reference's fuzzing corpus (tests/dav1d-test-data/oss-fuzz/
{asan,msan,ubsan}: clusterfuzz inputs that once crashed dav1d, copied as data into
tests/golden/oss_fuzz/): every input must end in events or -errno returns, never a crash, a hang
or an unbounded allocation (8 GiB address-space limit), as the reference's fuzz tests require of
dav1d (tests/libfuzzer/dav1d_fuzzer.c)."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CORPUS = os.path.join(HERE, "golden", "oss_fuzz")


@pytest.mark.parametrize("threads", [1, 4])
def test_fuzz_corpus_never_crashes(threads):
    """threads 4: the front-end's frame threads, failures surfacing from worker threads."""
    names = sorted(os.listdir(CORPUS))
    assert len(names) >= 100
    r = subprocess.run([sys.executable, os.path.join(HERE, "fuzz_child.py"), CORPUS, str(threads)],
                       capture_output=True, text=True, timeout=600)
    done = [ln.split()[0] for ln in r.stdout.splitlines() if ln.strip()]
    assert r.returncode == 0, f"front-end died (rc {r.returncode}) after {done[-1:]}: {r.stderr[-500:]}"
    assert done == names
