// Experiment (NOT part of libgnnrec): host builder of the panel-stepped edge streams for
// tools/exp_tiled.hip (v2). g++ -O3 -fopenmp -shared -fPIC.
//
// Block b = destination rows [b*R, min(N, (b+1)*R)) (one persistent workgroup at a time,
// accumulators in LDS). Its edges are cut by source-column panel (col / Wp); a step = one
// panel with edges in the block. Inside a step the rows are dealt to the NW waves by LPT on
// their edge counts in that panel (any wave may own a row in a step: steps are separated by a
// workgroup barrier), and each wave's rows are laid back to back into chunks of CH slots (a
// row's edges of the panel are a run in column order; a slot continuing a run inside the same
// chunk chains on the previous slot's new value). Unused slots are dummies (row = R scratch,
// val = 0, xoff of the chunk's first slot).
//
// Output per (block, wave): a contiguous chunk list (blocks major, waves minor), each slot
//   xoff uint32 (col * row_bytes), val f32, meta uint16 = row (10 bits) | bar << 10 | chain << 15,
// where bar (slot 0 only, 5 bits) = workgroup barriers to execute before the chunk.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>
#include <cstdlib>

namespace {

struct Entry {
  int32_t p, row;     // panel, local row
  int64_t k;          // first edge
  int32_t n;          // edges in this panel
};

struct BlockOut {
  std::vector<std::vector<uint32_t>> xoff;  // per wave
  std::vector<std::vector<float>> val;
  std::vector<std::vector<uint16_t>> meta;
  int32_t nsteps = 0;
};

struct Plan {
  int64_t n_blocks;
  int NW, CH;
  std::vector<BlockOut> blocks;
};

constexpr int kMaxBar = 31;

void build_block(const int64_t* rp, const int32_t* col, const float* val, int64_t N, int R,
                 int Wp, int NW, int CH, int64_t row_bytes, int64_t b, BlockOut& out) {
  static const int sub = getenv("EXP_SUB") ? atoi(getenv("EXP_SUB")) : 0;
  const int64_t r0 = b * R, r1 = std::min<int64_t>(N, r0 + R);
  std::vector<Entry> ent;
  for (int64_t r = r0; r < r1; ++r) {
    int64_t k = rp[r];
    const int64_t e = rp[r + 1];
    while (k < e) {
      const int32_t p = col[k] / Wp;
      int64_t j = k;
      while (j < e && col[j] / Wp == p) ++j;
      ent.push_back({p, (int32_t)(r - r0), k, (int32_t)(j - k)});
      k = j;
    }
  }
  std::stable_sort(ent.begin(), ent.end(), [](const Entry& a, const Entry& c) { return a.p < c.p; });
  out.xoff.assign(NW, {});
  out.val.assign(NW, {});
  out.meta.assign(NW, {});
  std::vector<int32_t> cur(NW, 0);   // step index of each wave's last emitted chunk
  int32_t step = 0;
  std::vector<int64_t> load(NW);
  std::vector<std::vector<const Entry*>> wl(NW);
  size_t i = 0;
  while (i < ent.size()) {
    size_t j = i;
    while (j < ent.size() && ent[j].p == ent[i].p) ++j;
    // LPT: largest count first onto the least loaded wave
    std::vector<const Entry*> g;
    for (size_t q = i; q < j; ++q) g.push_back(&ent[q]);
    std::stable_sort(g.begin(), g.end(), [](const Entry* a, const Entry* c) { return a->n > c->n; });
    std::fill(load.begin(), load.end(), 0);
    for (auto& v : wl) v.clear();
    for (const Entry* e : g) {
      int w = 0;
      for (int q = 1; q < NW; ++q)
        if (load[q] < load[w]) w = q;
      load[w] += e->n;
      wl[w].push_back(e);
    }
    for (int w = 0; w < NW; ++w) {
      if (wl[w].empty()) continue;
      // the wave's rows back to back (each row's edges a run in column order); a slot whose
      // row equals the previous slot's in the same chunk chains on that slot's new value
      std::vector<std::pair<const Entry*, int>> slots;
      for (const Entry* e : wl[w])
        for (int t = 0; t < e->n; ++t) slots.push_back({e, t});
      if (sub > 0)   // column sub-panels in ascending order inside the step (rows keep order)
        std::stable_sort(slots.begin(), slots.end(), [&](const std::pair<const Entry*, int>& a,
                                                         const std::pair<const Entry*, int>& c) {
          const int32_t ka = col[a.first->k + a.second] / sub, kc = col[c.first->k + c.second] / sub;
          if (ka != kc) return ka < kc;
          return a.first->row < c.first->row;
        });
      // chunking: a row may appear in a chunk only as one contiguous run (the kernel reads all
      // accumulators at the chunk start); a slot that would repeat a row non-adjacently is
      // deferred to a later chunk together with that row's later slots (per-row order kept)
      std::vector<std::pair<const Entry*, int>> seq;   // padded to chunks; first == null: dummy
      {
        std::vector<std::pair<const Entry*, int>> pending = slots, deferred;
        std::vector<int> in_chunk;
        std::vector<int> blocked;
        while (!pending.empty()) {
          deferred.clear();
          in_chunk.clear();
          blocked.clear();
          int n = 0, last = -1;
          const size_t start = seq.size();
          for (const auto& sl : pending) {
            const int r = sl.first->row;
            const bool is_blocked = std::find(blocked.begin(), blocked.end(), r) != blocked.end();
            const bool seen = std::find(in_chunk.begin(), in_chunk.end(), r) != in_chunk.end();
            if (n == CH || is_blocked || (seen && r != last)) {
              if (seen && r != last && !is_blocked) blocked.push_back(r);
              deferred.push_back(sl);
              continue;
            }
            seq.push_back(sl);
            if (!seen) in_chunk.push_back(r);
            last = r;
            ++n;
          }
          while (seq.size() - start < (size_t)CH) seq.push_back({nullptr, 0});
          pending.swap(deferred);
        }
      }
      const int C = (int)(seq.size() / CH);
      int32_t bar = step - cur[w];
      for (int c = 0; c < C; ++c) {
        while (bar > kMaxBar) {   // more barriers than the field holds: an empty chunk
          for (int s = 0; s < CH; ++s) {
            out.xoff[w].push_back(0);
            out.val[w].push_back(0.f);
            out.meta[w].push_back((uint16_t)(R | (s == 0 ? kMaxBar << 10 : 0)));
          }
          bar -= kMaxBar;
        }
        const size_t base = (size_t)c * CH;
        const int64_t k0 = seq[base].first->k + seq[base].second;
        const uint32_t x0 = (uint32_t)(col[k0] * row_bytes);
        for (int s = 0; s < CH; ++s) {
          uint32_t xo = x0;
          float v = 0.f;
          int row = R, chain = 0;
          const auto& sl = seq[base + s];
          if (sl.first) {
            const int64_t k = sl.first->k + sl.second;
            xo = (uint32_t)(col[k] * row_bytes);
            v = val[k];
            row = sl.first->row;
            chain = (s > 0 && seq[base + s - 1].first == sl.first) ? 1 : 0;
          }
          out.xoff[w].push_back(xo);
          out.val[w].push_back(v);
          out.meta[w].push_back((uint16_t)(row | (s == 0 ? bar << 10 : 0) | (chain << 15)));
        }
        bar = 0;
      }
      cur[w] = step;
    }
    ++step;
    i = j;
  }
  out.nsteps = step;
}

}  // namespace

extern "C" void* tiled_build(const int64_t* rp, const int32_t* col, const float* val, int64_t N,
                             int R, int Wp, int NW, int CH, int64_t row_bytes, int64_t* total,
                             int64_t* n_blocks) {
  auto* pl = new Plan;
  pl->n_blocks = (N + R - 1) / R;
  pl->NW = NW;
  pl->CH = CH;
  pl->blocks.resize(pl->n_blocks);
#pragma omp parallel for schedule(dynamic, 4)
  for (int64_t b = 0; b < pl->n_blocks; ++b)
    build_block(rp, col, val, N, R, Wp, NW, CH, row_bytes, b, pl->blocks[b]);
  int64_t t = 0;
  for (auto& bo : pl->blocks)
    for (int w = 0; w < NW; ++w) t += (int64_t)bo.xoff[w].size();
  *total = t;
  *n_blocks = pl->n_blocks;
  return pl;
}

// wptr [n_blocks*NW + 1] slot offsets; nsteps [n_blocks]
extern "C" void tiled_emit(void* h, uint32_t* xoff, float* val, uint16_t* meta, int64_t* wptr,
                           int32_t* nsteps) {
  auto* pl = static_cast<Plan*>(h);
  const int NW = pl->NW;
  std::vector<int64_t> off(pl->n_blocks * NW + 1, 0);
  for (int64_t b = 0; b < pl->n_blocks; ++b)
    for (int w = 0; w < NW; ++w)
      off[b * NW + w + 1] = off[b * NW + w] + (int64_t)pl->blocks[b].xoff[w].size();
  std::memcpy(wptr, off.data(), off.size() * sizeof(int64_t));
#pragma omp parallel for schedule(dynamic, 4)
  for (int64_t b = 0; b < pl->n_blocks; ++b) {
    nsteps[b] = pl->blocks[b].nsteps;
    for (int w = 0; w < NW; ++w) {
      const int64_t o = off[b * NW + w];
      const auto& bo = pl->blocks[b];
      std::memcpy(xoff + o, bo.xoff[w].data(), bo.xoff[w].size() * 4);
      std::memcpy(val + o, bo.val[w].data(), bo.val[w].size() * 4);
      std::memcpy(meta + o, bo.meta[w].data(), bo.meta[w].size() * 2);
    }
  }
}

extern "C" void tiled_free(void* h) { delete static_cast<Plan*>(h); }
