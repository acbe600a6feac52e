"""Child process of tests/test_fuzz_frontend.py: every input of the given directory through the
front-end (rav1d_amd/libmi_av1dec.so) in the reference fuzzer's framing
(tests/libfuzzer/dav1d_fuzzer.c: a 32-byte header, then frames of u32 size + u64 timestamp),
under an address-space limit. Prints one line per input; a crash kills this process, not the
test runner."""
import os
import resource
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def frames(data):
    off = 32
    while off + 12 <= len(data):
        size = struct.unpack_from("<I", data, off)[0]
        off += 12
        if size > len(data) or off + size > len(data):
            return
        if size:
            yield data[off:off + size]
        off += size


def main(d, threads):
    if not os.environ.get("FUZZ_NO_AS_LIMIT"):     # (AddressSanitizer reserves terabytes of shadow)
        resource.setrlimit(resource.RLIMIT_AS, (8 << 30, 8 << 30))
    from rav1d_amd.av1dec import Av1Decoder
    for name in sorted(os.listdir(d)):
        data = open(os.path.join(d, name), "rb").read()
        # one decoder for the whole input, fed on after every rejected temporal unit, as the
        # reference fuzzer keeps its context after a dav1d_send_data / dav1d_get_picture error
        # (tests/libfuzzer/dav1d_fuzzer.c:165-181): the front-end's recovery state is exercised
        dec, nev, nerr = Av1Decoder(threads), 0, 0
        for f in frames(data):
            try:
                dec.send(f)
            except RuntimeError:
                nerr += 1
            try:
                for _ in dec.events():
                    nev += 1
            except RuntimeError:
                nerr += 1
        try:
            for _ in dec.events():
                nev += 1
        except RuntimeError:
            nerr += 1
        print(name, nev, nerr, flush=True)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1)
