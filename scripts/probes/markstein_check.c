#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <math.h>
#include <string.h>
#include <omp.h>
static inline uint64_t rnd(uint64_t *s) { uint64_t x = *s; x ^= x << 13; x ^= x >> 7; x ^= x << 17; return *s = x; }
static inline float fbits(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t ubits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float mk(float a, float b, float y) { float q = a * y; float r = fmaf(-q, b, a); return fmaf(r, y, q); }
int main(int argc, char **argv) {
    long n = atol(argv[1]); long bad = 0, tested = 0;
#pragma omp parallel reduction(+:bad,tested)
    {
        uint64_t s = 88172645463325252ull * (omp_get_thread_num() + 1);
#pragma omp for
        for (long i = 0; i < n; ++i) {
            /* b: random exponent in [-60, 60], sign random; midpoint target with random exponent offset */
            uint32_t eb = 127 - 60 + (uint32_t)(rnd(&s) % 121);
            float b = fbits((uint32_t)(rnd(&s) & 0x80000000u) | (eb << 23) | (uint32_t)(rnd(&s) & 0x7FFFFF));
            uint32_t eq = 127 - 40 + (uint32_t)(rnd(&s) % 81);
            float f1 = fbits((eq << 23) | (uint32_t)(rnd(&s) & 0x7FFFFF));
            double mu = ((double)f1 + (double)fbits(ubits(f1) + 1)) / 2.0;
            float a0 = (float)((double)b * mu);
            float y = 1.0f / b;
            for (int k = -4; k <= 4; ++k) {
                float a = fbits(ubits(a0) + k);
                uint32_t ea = (ubits(a) >> 23) & 0xFF;
                if (ea < 67 || ea > 187) continue;
                float ref = a / b, got = mk(a, b, y);
                ++tested;
                if (ubits(ref) != ubits(got)) { if (bad < 10) printf("a=%a b=%a ref=%a got=%a\n", a, b, ref, got); ++bad; }
            }
            uint32_t ea = 127 - 60 + (uint32_t)(rnd(&s) % 121);
            float a = fbits((uint32_t)(rnd(&s) & 0x80000000u) | (ea << 23) | (uint32_t)(rnd(&s) & 0x7FFFFF));
            float ref = a / b, got = mk(a, b, y); ++tested;
            if (ubits(ref) != ubits(got)) { if (bad < 10) printf("R a=%a b=%a ref=%a got=%a\n", a, b, ref, got); ++bad; }
        }
    }
    printf("tested %ld bad %ld\n", tested, bad);
    return 0;
}
