// fingerprint.hpp -- 128-bit state fingerprint and the HBM-resident visited table.
//
// Fingerprint: MurmurHash3_x64_128 block/finalizer structure over the canonical packed
// state (16-byte blocks, the state width is a multiple of 16 bytes). Unused bits of a
// packed state are always zero, so equal canonical states have equal fingerprints.
//
// Visited table: open addressing over 8-byte slots in 64-byte buckets. A slot holds the
// fingerprint's high word with bit 0 forced to 1 (non-zero), i.e. 63 bits of it; the home slot
// is taken from the low word (bucket: its low bits, slot in the bucket: bits 28-30) and the
// owner shard (multi-GPU) from its top bits, so a stored key pins 63 + log2(buckets) +
// log2(shards) bits of the 128-bit fingerprint. Slots are write-once (0 -> key with one 64-bit
// CAS): no two-phase publish, no spinning on another lane's store.
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

struct Table {
  unsigned long long* slots;  // nbuckets * 8
  uint64_t bucket_mask;       // nbuckets - 1 (power of two)
  int max_probes;             // buckets visited before declaring the table full
};

#ifndef DSL_TABLE_LOAD_FIRST
// The probe IS the insert. Slots are visited linearly from a home slot inside the home bucket; a
// CAS(0 -> key) per slot answers both questions at once (old == 0: inserted; old == key: present;
// else the next slot). Write-once slots make this exact: a key lies at or after its home slot with
// no empty slot in between, so an empty slot reached first means "absent". Agent-scope atomics
// are performed at the memory side (coherent across the 8 XCD L2s), so a probe is ONE memory
// round trip whether the state is new or not -- a bucket load followed by a CAS was two for every
// new state (measured on C5: +18 % at d12, +26 % at d14, profiles/r02_*).
__device__ __forceinline__ uint64_t table_home(const Table& t, const Fp& f) {
  return ((f.lo & t.bucket_mask) << 3) | ((f.lo >> 28) & 7);
}
// The CAS at the home slot, issued now and answered later (table_settle): work placed in between
// runs while the atomic is in flight.
__device__ __forceinline__ unsigned long long table_cas_home(const Table& t, const Fp& f) {
  return atomicCAS(t.slots + table_home(t, f), 0ull, (unsigned long long)(f.hi | 1ull));
}
__device__ __forceinline__ int table_settle(const Table& t, const Fp& f, unsigned long long old) {
  const unsigned long long key = (unsigned long long)(f.hi | 1ull);
  if (old == 0ull) return INS_NEW;
  if (old == key) return INS_EXISTS;
  const uint64_t nmask = t.bucket_mask * 8 + 7;
  uint64_t i = table_home(t, f);
  for (int probe = 1; probe < 8 * t.max_probes; probe++) {
    i = (i + 1) & nmask;
    old = atomicCAS(t.slots + i, 0ull, key);
    if (old == 0ull) return INS_NEW;
    if (old == key) return INS_EXISTS;
  }
  return INS_FULL;
}
__device__ __forceinline__ int table_insert(const Table& t, const Fp& f) { return table_settle(t, f, table_cas_home(t, f)); }
#else  // DSL_TABLE_LOAD_FIRST: read the bucket line, CAS only into an empty slot (round 1)
__device__ __forceinline__ int table_insert(const Table& t, const Fp& f) {
  const unsigned long long key = (unsigned long long)(f.hi | 1ull);
  uint64_t b = f.lo & t.bucket_mask;
  for (int probe = 0; probe < t.max_probes; probe++) {
    unsigned long long* B = t.slots + ((b + (uint64_t)probe) & t.bucket_mask) * 8;
    // One 64-byte line: four 16-byte loads.
    const ulonglong2* B2 = reinterpret_cast<const ulonglong2*>(B);
    ulonglong2 q0 = B2[0], q1 = B2[1], q2 = B2[2], q3 = B2[3];
    unsigned long long s[8] = {q0.x, q0.y, q1.x, q1.y, q2.x, q2.y, q3.x, q3.y};
    bool hit = false;
#pragma unroll
    for (int j = 0; j < 8; j++) hit |= (s[j] == key);
    if (hit) return INS_EXISTS;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if (s[j] != 0) continue;  // occupied by another key (write-once)
      unsigned long long old = atomicCAS(B + j, 0ull, key);
      if (old == 0ull) return INS_NEW;
      if (old == key) return INS_EXISTS;
    }
  }
  return INS_FULL;
}
#endif

}  // namespace dsl
