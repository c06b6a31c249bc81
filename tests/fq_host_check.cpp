// Host check of plonky3_eon_amd/csrc/fq_host.h (tests/test_fq_host.py): reads 256-bit inputs as
// four comma-separated hex 64-bit limbs per line (little-endian) from stdin and prints
// inverse(a) and mul(a, a) in the same form.
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "fq_host.h"

using namespace eon::hostq;

int main() {
    char line[512];
    while (std::fgets(line, sizeof line, stdin)) {
        F a;
        char* p = line;
        for (int i = 0; i < 4; i++) {
            a.l[i] = std::strtoull(p, &p, 16);
            if (*p == ',') p++;
        }
        const F inv = inverse(a), sq = mul(a, a);
        std::printf("%llx,%llx,%llx,%llx %llx,%llx,%llx,%llx\n", (unsigned long long)inv.l[0],
                    (unsigned long long)inv.l[1], (unsigned long long)inv.l[2], (unsigned long long)inv.l[3],
                    (unsigned long long)sq.l[0], (unsigned long long)sq.l[1], (unsigned long long)sq.l[2],
                    (unsigned long long)sq.l[3]);
    }
    return 0;
}
