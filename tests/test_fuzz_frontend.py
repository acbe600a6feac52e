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


def test_fuzz_corpus_under_address_sanitizer(tmp_path):
    """The same corpus through an ASan + UBSan build of the front-end (host code: the GPU has
    no sanitizer here), one decoder per input fed on across errors: an out-of-bounds access
    or undefined behaviour that the -O3 build survives silently fails here."""
    import shutil
    asan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    if not asan or not os.path.exists(asan) or not shutil.which("make"):
        pytest.skip("no libasan")
    out = tmp_path / "libmi_av1dec_asan.so"
    r = subprocess.run(["make", "-s", "-j8", "-C", os.path.join(os.path.dirname(HERE), "rav1d_amd", "host"), "asan",
                        f"ASAN_OUT={out}"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    env = dict(os.environ, MI_DEC_LIB=str(out), LD_PRELOAD=os.path.realpath(asan), FUZZ_NO_AS_LIMIT="1",
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([sys.executable, os.path.join(HERE, "fuzz_child.py"), CORPUS, "1"], env=env,
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, (r.stdout[-1000:], r.stderr[-3000:])
    assert len(r.stdout.splitlines()) == len(os.listdir(CORPUS))
