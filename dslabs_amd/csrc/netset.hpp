// netset.hpp -- the network as a canonical bounded SET of 32-bit message records.
//
// SearchState keeps every sent message forever; delivery never removes, duplicates collapse
// (SearchState.java:71, :300-301; labs/lab0-pingpong/README.md:485-494). Protocols whose message
// universe is too large for a bitmap store the set as a sorted, duplicate-free array of
// records in a fixed region of the packed state: word `base` holds the count, words
// base+1 .. base+CAP the records in ascending order, unused words zero.
#pragma once
#include "common.hpp"

namespace dsl {

template <int BASE, int CAP>
struct NetSet {
  template <class S>
  static DSL_HD int size(const S& s) {
    return (int)s.w[BASE];
  }
  template <class S>
  static DSL_HD uint32_t at(const S& s, int i) {
    return s.w[BASE + 1 + i];
  }
  // Returns 0 inserted, 1 already present, -1 overflow (caller reports STEP_OVERFLOW).
  template <class S>
  static DSL_HD int insert(S& s, uint32_t rec) {
    int n = (int)s.w[BASE];
    int pos = 0;
    while (pos < n && s.w[BASE + 1 + pos] < rec) pos++;
    if (pos < n && s.w[BASE + 1 + pos] == rec) return 1;
    if (n >= CAP) return -1;
    for (int j = n; j > pos; j--) s.w[BASE + 1 + j] = s.w[BASE + j];
    s.w[BASE + 1 + pos] = rec;
    s.w[BASE] = (uint32_t)(n + 1);
    return 0;
  }
};

}  // namespace dsl
