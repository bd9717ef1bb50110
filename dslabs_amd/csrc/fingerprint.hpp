// fingerprint.hpp -- 128-bit state fingerprint and the HBM-resident visited table.
//
// Fingerprint: MurmurHash3_x64_128 block/finalizer structure over the canonical packed
// state (16-byte blocks, the state width is a multiple of 16 bytes). Unused bits of a
// packed state are always zero, so equal canonical states have equal fingerprints.
//
// Visited table (the BFS `discovered` set, Search.java:406-408): open addressing over 8-byte
// slots in 64-byte buckets, linear probing from a home slot; slots are write-once (0 -> key with
// one 64-bit CAS: no two-phase publish, no spinning on another lane's store). It GROWS: at a level
// boundary the table is rehashed into a larger one (k_rehash), so a stored key carries what its
// new home needs (see table_key0).
#pragma once
#include "common.hpp"

namespace dsl {

struct Fp {
  uint64_t hi, lo;
};

DSL_HD uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
DSL_HD uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

template <int W>
DSL_HD Fp fingerprint(const uint32_t (&w)[W]) {
  static_assert(W % 4 == 0, "packed state must be a multiple of 16 bytes");
  const uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
  uint64_t h1 = 0x9368e53c2f6af274ULL, h2 = 0x586dcd208f7cd3fdULL;
#pragma unroll
  for (int i = 0; i < W; i += 4) {
    uint64_t k1 = (uint64_t)w[i] | ((uint64_t)w[i + 1] << 32);
    uint64_t k2 = (uint64_t)w[i + 2] | ((uint64_t)w[i + 3] << 32);
    k1 *= c1;
    k1 = rotl64(k1, 31);
    k1 *= c2;
    h1 ^= k1;
    h1 = rotl64(h1, 27);
    h1 += h2;
    h1 = h1 * 5 + 0x52dce729;
    k2 *= c2;
    k2 = rotl64(k2, 33);
    k2 *= c1;
    h2 ^= k2;
    h2 = rotl64(h2, 31);
    h2 += h1;
    h2 = h2 * 5 + 0x38495ab5;
  }
  h1 ^= (uint64_t)(W * 4);
  h2 ^= (uint64_t)(W * 4);
  h1 += h2;
  h2 += h1;
  h1 = fmix64(h1);
  h2 = fmix64(h2);
  h1 += h2;
  h2 += h1;
  return Fp{h1, h2};
}

// Owner shard of a fingerprint: multiply-shift on the top 32 bits of the low word.
DSL_HD int owner_of(const Fp& f, int world) {
  return (int)(((f.lo >> 32) * (uint64_t)world) >> 32);
}

enum InsertRc : int { INS_NEW = 0, INS_EXISTS = 1, INS_FULL = 2 };

// A table of 2^b buckets (b = log2(bucket_mask + 1)). Home bucket = lo & bucket_mask, first slot
// in it = the top 3 bits of hi. Slot word: bit 0 = 1 (never 0); bits 1-3 = the bucket
// displacement d of the slot from its home bucket (probing stops past kMaxDisp buckets); bits
// 4 .. 4+g-1 = lo bits [b0, b0 + g), the home-bucket bits of every larger table (b0 = log2 of the
// search's first table, g = kKeyBits - b0); above them hi's bits from 4 + g up. A slot's home is
// therefore recomputable from the slot alone -- its bucket minus d, plus the bits the larger table
// needs -- and a stored key pins (60 - g) + b + (g - (b - b0)) = 60 + b0 bits of the fingerprint
// (77 at the default first table of 2^20 slots): n distinct states merge with probability about
// n^2 / 2^(61 + b0). The owner shard (top 32 bits of lo) is disjoint from the home bits.
constexpr int kKeyBits = 32;  // home-bucket bits of the largest table (2^32 buckets = 2^35 slots)
constexpr int kMaxDisp = 7;   // buckets a key may sit past its home bucket

struct Table {
  unsigned long long* slots;  // nbuckets * 8
  uint64_t bucket_mask;       // nbuckets - 1 (power of two)
  int32_t b0;                 // log2(buckets) of the search's first table: the key layout
  int32_t load_first;         // probe by a load first, CAS only an empty slot (table_insert)
};

DSL_HD uint64_t table_key0(const Table& t, const Fp& f) {
  const int g = kKeyBits - t.b0;
  const uint64_t lo_bits = ((f.lo >> t.b0) & ((1ull << g) - 1ull)) << 4;
  return (f.hi & ~((1ull << (g + 4)) - 1ull)) | lo_bits | 1ull;
}
DSL_HD uint64_t table_home(const Table& t, const Fp& f) { return ((f.lo & t.bucket_mask) << 3) | (f.hi >> 61); }

// The probe IS the insert. Slots are visited linearly from the home slot; a CAS(0 -> key) per
// slot answers both questions at once (old == 0: inserted; old == key: present; else the next
// slot). Write-once slots make this exact: a key lies at or after its home slot with no empty slot
// in between, so an empty slot reached first means "absent" (a slot's word includes its
// displacement, the same for every probe of one fingerprint). Agent-scope atomics are performed at
// the memory side (coherent across the 8 XCD L2s), so a probe is ONE memory round trip whether the
// state is new or not (a bucket load followed by a CAS was two for every new state: +18 % at d12,
// +26 % at d14 on C5, profiles/r02_*).
//
// load_first (a table far beyond the Infinity Cache, where probes are bound by the memory-side
// atomic rate rather than latency): each slot is read with a plain load first and only an empty
// one is CAS'd. A load can only be stale towards 0 (slots are write-once), which the CAS then
// corrects, so the answer is the same; a state already present costs a read instead of an atomic.
// first > 0: the probe continues at slot home + first (the earlier slots were CAS'd and held other
// keys; k_level's judge-overlap variant issues the home slot's CAS itself)
__device__ __forceinline__ int table_insert(const Table& t, const Fp& f, int first = 0) {
  const uint64_t k0 = table_key0(t, f), home = table_home(t, f), nmask = t.bucket_mask * 8 + 7;
  uint64_t i = (home + (uint64_t)first) & nmask;
  for (int probe = first; probe < 8 * (kMaxDisp + 1); probe++) {
    const uint64_t d = ((i >> 3) - (home >> 3)) & t.bucket_mask;
    if (d > (uint64_t)kMaxDisp) break;
    const unsigned long long key = (unsigned long long)(k0 | (d << 1));
    unsigned long long old = 0ull;
    if (t.load_first) old = __hip_atomic_load(t.slots + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == 0ull) {
      old = atomicCAS(t.slots + i, 0ull, key);
      if (old == 0ull) return INS_NEW;
    }
    if (old == key) return INS_EXISTS;
    i = (i + 1) & nmask;
  }
  return INS_FULL;
}

// The home slot, in the larger table `to` (same b0), of slot word v found at slot index i of
// `from`: its home bucket in `from` is its bucket minus its displacement; the larger table's
// extra home bits are the key's stored lo bits.
DSL_HD uint64_t table_rehome(const Table& from, const Table& to, uint64_t i, uint64_t v) {
  const uint64_t d = (v >> 1) & 7ull;
  const uint64_t hb = ((i >> 3) - d) & from.bucket_mask;
  int b = 0;
  while ((2ull << b) <= from.bucket_mask + 1) b++;  // log2(buckets of `from`)
  const uint64_t extra = ((v >> 4) >> (b - from.b0)) << b;  // lo bits [b, b0 + g) at their place
  return (((hb | extra) & to.bucket_mask) << 3) | (v >> 61);
}

}  // namespace dsl
