// Document placement for data-parallel LDA: longest-processing-time
// greedy of the heavy documents over the ranks, on top of the hash load of all other documents.
//
// The reference shipped whole corpus files to MPI ranks (oni-lda-c, [U-H]); here documents are
// IPs with a power-law token count, so a handful of them would otherwise pin one rank. The greedy
// runs once per day over at most HEAVY_DOCS_PER_RANK × world candidates (oni355/pipeline/common.py
// place_docs); in Python it cost tens of milliseconds inside the timed day, here microseconds.
#include "oni_native.h"

// counts[n]: candidate token counts, already in placement order (count desc, key asc).
// load[W] (in/out): per-rank token load before/after placement. owner[n] (out): rank of each
// candidate. Ties go to the lowest rank, so every rank computes the same placement.
ONI_NATIVE_API int oni_lpt_place(const int64_t* counts, int64_t n, int32_t W, int64_t* load, int32_t* owner) {
  if (W <= 0 || n < 0 || (n > 0 && (!counts || !owner)) || !load) return 1;
  for (int64_t i = 0; i < n; ++i) {
    int32_t best = 0;
    for (int32_t r = 1; r < W; ++r)
      if (load[r] < load[best]) best = r;
    load[best] += counts[i];
    owner[i] = best;
  }
  return 0;
}
