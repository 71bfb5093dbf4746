/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into or called by the product
 * (flpytorch_amd/).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it, and only as the checker.
 *
 * Plain-C restatement of the numpy *legacy* MT19937 stream (NEP 19 frozen) that
 * FL_PyTorch draws every compressor pattern from: the experiment-wide
 * np.random.RandomState (fl_pytorch/utils/execution_context.py:25).  Third-party
 * dependency: numpy (unpinned in the reference, requirements.txt:6); the container's
 * numpy 2.2.6 produced the pinning fixtures tests/golden/rng.npz.
 *
 * Restated published algorithms:
 *   - MT19937 init_genrand / twist / tempering (Matsumoto & Nishimura 1998),
 *     the seeding numpy's RandomState(int) uses;
 *   - legacy random_interval(max): draws next_uint32 & mask until <= max;
 *   - legacy shuffle: for i = n-1 .. 1: j = random_interval(i); swap(a[i], a[j]);
 *     choice(n, k, replace=False) == permutation(n)[:k]   (compressors.py:206,
 *     fl_funcs.py:15);
 *   - random_sample: ((a >> 5) * 2^26 + (b >> 6)) / 2^53   (compressors.py:204, 208-212);
 *   - randint(2**31): one masked draw next_uint32 & 0x7FFFFFFF (algorithms.py:2055).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define MT_N 624
#define MT_M 397

typedef struct {
    uint32_t key[MT_N];
    int pos;
} orc_mt;

void orc_mt_seed(orc_mt *s, uint32_t seed) {
    s->key[0] = seed;
    for (int i = 1; i < MT_N; i++)
        s->key[i] = 1812433253u * (s->key[i - 1] ^ (s->key[i - 1] >> 30)) + (uint32_t)i;
    s->pos = MT_N;
}

static void orc_twist(orc_mt *s) {
    for (int i = 0; i < MT_N; i++) {
        uint32_t y = (s->key[i] & 0x80000000u) | (s->key[(i + 1) % MT_N] & 0x7fffffffu);
        s->key[i] = s->key[(i + MT_M) % MT_N] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    s->pos = 0;
}

uint32_t orc_mt_next32(orc_mt *s) {
    if (s->pos >= MT_N) orc_twist(s);
    uint32_t y = s->key[s->pos++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

double orc_mt_next_double(orc_mt *s) {
    uint32_t a = orc_mt_next32(s) >> 5, b = orc_mt_next32(s) >> 6;
    return (a * 67108864.0 + b) / 9007199254740992.0;
}

static uint64_t orc_interval(orc_mt *s, uint64_t max) {
    if (max == 0) return 0;
    uint64_t mask = max;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4;
    mask |= mask >> 8; mask |= mask >> 16; mask |= mask >> 32;
    uint64_t v;
    if (max <= 0xffffffffull) {
        while ((v = (orc_mt_next32(s) & mask)) > max) {}
    } else {
        do {
            uint64_t hi = orc_mt_next32(s), lo = orc_mt_next32(s);
            v = ((hi << 32) | lo) & mask;
        } while (v > max);
    }
    return v;
}

/* choice(n, k, replace=False) -> out[k] ; scratch perm[n] (caller-sized) */
void orc_mt_choice(orc_mt *s, int64_t n, int64_t k, int64_t *out, int64_t *perm) {
    for (int64_t i = 0; i < n; i++) perm[i] = i;
    for (int64_t i = n - 1; i >= 1; i--) {
        int64_t j = (int64_t)orc_interval(s, (uint64_t)i);
        int64_t t = perm[i]; perm[i] = perm[j]; perm[j] = t;
    }
    memcpy(out, perm, (size_t)k * sizeof(int64_t));
}

void orc_mt_rand(orc_mt *s, int64_t n, double *out) {
    for (int64_t i = 0; i < n; i++) out[i] = orc_mt_next_double(s);
}

int64_t orc_mt_randint31(orc_mt *s) { return (int64_t)(orc_mt_next32(s) & 0x7fffffffu); }

int orc_mt_state_size(void) { return (int)sizeof(orc_mt); }
