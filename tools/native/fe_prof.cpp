// Front-end profiling driver (diagnostic, not shipped): decodes IVF streams through the C API
// of libmi_av1dec (include/mi_av1dec.h) on one thread, REPS times, and prints the wall time per
// pass. Built with the front-end's sources and -pg by tools/native/Makefile, for gprof.
//   fe_prof FILE.ivf [REPS]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "mi_av1dec.h"

int main(int argc, char **argv) {
    if (argc < 2) return 2;
    FILE *fp = fopen(argv[1], "rb");
    if (!fp) return 2;
    std::vector<uint8_t> d;
    uint8_t buf[1 << 16];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, fp)) > 0) d.insert(d.end(), buf, buf + n);
    fclose(fp);
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    if (d.size() < 32 || d[0] != 'D') return 2;
    for (int r = 0; r < reps; r++) {
        const auto t0 = std::chrono::steady_clock::now();
        MiDec *dec = nullptr;
        if (mi_dec_create(&dec)) return 1;
        size_t p = 32;
        int frames = 0;
        while (p + 12 <= d.size()) {
            const uint32_t sz = d[p] | d[p + 1] << 8 | d[p + 2] << 16 | (uint32_t)d[p + 3] << 24;
            p += 12;
            if (p + sz > d.size()) break;
            if (mi_dec_send(dec, d.data() + p, sz)) { fprintf(stderr, "%s\n", mi_dec_error(dec)); return 1; }
            p += sz;
            MiDecEvent ev;
            int k;
            while ((k = mi_dec_next(dec, &ev)) == 1) frames += ev.frame != nullptr;
            if (k < 0) { fprintf(stderr, "%s\n", mi_dec_error(dec)); return 1; }
        }
        mi_dec_destroy(dec);
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        printf("pass %d: %d frames %.2f ms\n", r, frames, ms);
    }
    return 0;
}
