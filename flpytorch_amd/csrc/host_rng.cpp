// Host side of compat mode: the numpy legacy MT19937 stream the reference draws every pattern
// from (np.random.RandomState, fl_pytorch/utils/execution_context.py:25), advanced in place on
// the caller's (key[624], pos) state so the Python layer can hand it back with set_state().
//
//   flc_mt_choice    rndgen.choice(D, K, replace=False)   compressors.py:206 (== permutation(D)[:K],
//                    Fisher-Yates i = D-1..1, j = bounded draw by masked rejection)
//   flc_mt_rand      rndgen.rand(D)                       compressors.py:208-212 (53-bit doubles)
//   flc_mt_randint31 rndgen.randint(2**31)                algorithms.py:2055
//
// Throughput matters here (the reference's choice(1e6, 1e4) costs 24 ms per client): the
// generator refills 624 words per twist in a tight loop and the shuffle runs on a flat int64
// array.  The whole Fisher-Yates sweep is required: every swap can move a value into the first
// K slots, and every draw advances the shared stream.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "../../include/flcodec.h"
#include "common.hpp"
#include "randk_tree.hpp"

namespace {

struct Mt {
    uint32_t* key;
    int32_t* pos;
    uint32_t buf_;
    inline void twist() {
        constexpr uint32_t UP = 0x80000000u, LO = 0x7fffffffu, A = 0x9908b0dfu;
        int i = 0;
        for (; i < 624 - 397; ++i) {
            uint32_t y = (key[i] & UP) | (key[i + 1] & LO);
            key[i] = key[i + 397] ^ (y >> 1) ^ ((0u - (y & 1u)) & A);
        }
        for (; i < 623; ++i) {
            uint32_t y = (key[i] & UP) | (key[i + 1] & LO);
            key[i] = key[i + 397 - 624] ^ (y >> 1) ^ ((0u - (y & 1u)) & A);
        }
        uint32_t y = (key[623] & UP) | (key[0] & LO);
        key[623] = key[396] ^ (y >> 1) ^ ((0u - (y & 1u)) & A);
        *pos = 0;
    }
    inline uint32_t next() {
        if (*pos >= 624) twist();
        uint32_t y = key[(*pos)++];
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= (y >> 18);
        return y;
    }
    inline double next_double() {
        const uint32_t a = next() >> 5, b = next() >> 6;
        return (a * 67108864.0 + b) / 9007199254740992.0;
    }
    inline uint64_t bounded(uint64_t max) {   // legacy random_interval
        if (max == 0) return 0;
        uint64_t mask = max;
        mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4;
        mask |= mask >> 8; mask |= mask >> 16; mask |= mask >> 32;
        if (max <= 0xffffffffull) {
            const uint32_t m32 = (uint32_t)mask, mx = (uint32_t)max;
            uint32_t v;
            do { v = next() & m32; } while (v > mx);
            return v;
        }
        uint64_t v;
        do {
            const uint64_t hi = next();
            const uint64_t lo = next();
            v = ((hi << 32) | lo) & mask;
        } while (v > max);
        return v;
    }
};

bool valid_state(const uint32_t* key, const int32_t* pos) { return key && pos && *pos >= 0 && *pos <= 624; }

}  // namespace

extern "C" int flc_mt_choice(uint32_t* h_key, int32_t* h_pos, int64_t n, int64_t k, int64_t* h_out,
                             int64_t* h_scratch) {
    if (!valid_state(h_key, h_pos) || n < 0 || k < 0 || k > n || (k > 0 && !h_out) || (n > 0 && !h_scratch)) {
        flc::set_error("flc_mt_choice: bad arguments");
        return FLC_ERR_ARG;
    }
    Mt mt{h_key, h_pos, 0};
    int64_t* a = h_scratch;
    for (int64_t i = 0; i < n; ++i) a[i] = i;
    for (int64_t i = n - 1; i >= 1; --i) {
        const int64_t j = (int64_t)mt.bounded((uint64_t)i);
        const int64_t t = a[i];
        a[i] = a[j];
        a[j] = t;
    }
    memcpy(h_out, a, (size_t)k * sizeof(int64_t));
    return FLC_OK;
}

extern "C" int flc_mt_rand(uint32_t* h_key, int32_t* h_pos, int64_t n, double* h_out) {
    if (!valid_state(h_key, h_pos) || n < 0 || (n > 0 && !h_out)) {
        flc::set_error("flc_mt_rand: bad arguments");
        return FLC_ERR_ARG;
    }
    Mt mt{h_key, h_pos, 0};
    if (n == 0) return FLC_OK;
    // 1) sequential: the raw (untempered) words of the draws, block by block, parked in the
    //    output array itself (a pair of words occupies exactly the 8 bytes of its double).  The
    //    words are copied in stream order before each twist, so a pair that straddles the end of
    //    a 624-word block (any odd start position) needs no special case.
    uint32_t* raw = reinterpret_cast<uint32_t*>(h_out);
    const int64_t m_total = n;
    int64_t w = 0;
    while (w < 2 * m_total) {
        if (*h_pos >= 624) mt.twist();
        const int64_t take = std::min<int64_t>(624 - *h_pos, 2 * m_total - w);
        memcpy(raw + w, h_key + *h_pos, (size_t)take * sizeof(uint32_t));
        *h_pos += (int32_t)take;
        w += take;
    }
    // 2) parallel, in place: tempering and the 53-bit conversion (a * 2^26 + b) * 2^-53 (the
    //    reference's division by 2^53 is exact, so is the product)
    auto convert = [raw](int64_t t0, int64_t t1) {
        double* o = reinterpret_cast<double*>(raw);
        for (int64_t t = t0; t < t1; ++t) {
            uint32_t a = raw[2 * t], b = raw[2 * t + 1];
            a ^= (a >> 11); a ^= (a << 7) & 0x9d2c5680u; a ^= (a << 15) & 0xefc60000u; a ^= (a >> 18);
            b ^= (b >> 11); b ^= (b << 7) & 0x9d2c5680u; b ^= (b << 15) & 0xefc60000u; b ^= (b >> 18);
            o[t] = ((double)(int32_t)(a >> 5) * 67108864.0 + (double)(int32_t)(b >> 6)) * (1.0 / 9007199254740992.0);
        }
    };
    const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const int64_t per = (m_total + hw - 1) / hw;
    if (hw == 1 || m_total < (1 << 18)) {
        convert(0, m_total);
    } else {
        std::vector<std::thread> th;
        for (unsigned q = 0; q < hw; ++q) {
            const int64_t t0 = (int64_t)q * per, t1 = std::min<int64_t>(m_total, t0 + per);
            if (t0 < t1) th.emplace_back(convert, t0, t1);
        }
        for (auto& t : th) t.join();
    }
    return FLC_OK;
}

extern "C" int flc_mt_randint31(uint32_t* h_key, int32_t* h_pos, int64_t count, int64_t* h_out) {
    if (!valid_state(h_key, h_pos) || count < 0 || (count > 0 && !h_out)) {
        flc::set_error("flc_mt_randint31: bad arguments");
        return FLC_ERR_ARG;
    }
    Mt mt{h_key, h_pos, 0};
    for (int64_t i = 0; i < count; ++i) h_out[i] = (int64_t)(mt.next() & 0x7fffffffu);
    return FLC_OK;
}

extern "C" double flc_device_uniform(uint64_t seed, int64_t client, int64_t j) {
    return (double)flc::dev_u32(flc::client_key(seed, client), (uint32_t)j) * (1.0 / 4294967296.0);
}

extern "C" int flc_device_randk_indices(uint64_t seed, int64_t client, int64_t d, int64_t k, int64_t* h_out) {
    if (d < 1 || k < 0 || k > d || (k > 0 && !h_out)) {
        flc::set_error("flc_device_randk_indices: bad arguments");
        return FLC_ERR_ARG;
    }
    // host mirror of k_randk_counts (histogram of the row permutation's first k images by chunk)
    // + the chunk permutations: chunk by chunk, within a chunk in permutation order
    namespace rt = flc::rktree;
    const uint64_t ck = flc::client_key(seed, client);
    const int64_t C = (d + rt::CH - 1) / rt::CH;
    std::vector<int64_t> cnt((size_t)C, 0);
    const rt::RowPerm P(ck, (uint64_t)d);
    for (int64_t t = 0; t < k; ++t) ++cnt[(size_t)(P((uint64_t)t) >> rt::CH_SHIFT)];
    int64_t pos = 0;
    for (int64_t c = 0; c < C; ++c) {
        const uint32_t clen = (uint32_t)std::min<int64_t>(rt::CH, d - c * rt::CH);
        const rt::ChunkPerm Q(ck, c, clen);
        for (int64_t t = 0; t < cnt[(size_t)c]; ++t) h_out[pos++] = c * rt::CH + Q((uint32_t)t);
    }
    return pos == k ? FLC_OK : FLC_ERR_ARG;
}
