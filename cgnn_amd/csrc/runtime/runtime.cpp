// cgnn_amd._rt -- host C++ runtime (no GPU dependency, builds and runs on CPU).
//
//  * dag_program      compiles one causal DAG (+ optional confounder skeleton)
//                     into the int32 "DAG program" the HIP generator kernels
//                     execute (layout documented in engine/program.py).  The
//                     generation order reproduces the reference's sweep
//                     (CGNN.py:63-84): repeated passes over the variable list,
//                     emitting every variable whose parents are all generated.
//  * is_acyclic / topo_order / canonical_hash   graph algorithms used by the
//                     structure searches (fix for SURVEY §2.6 B11: hash of the
//                     sorted edge list instead of list-of-dict comparisons).
//  * csr_from_edges   parallel counting-sort CSR builder (optional symmetrise,
//                     self loops, duplicate removal).
//  * synthetic_graph  ogbn-shaped random graph with planted communities and a
//                     power-law-ish degree profile (Phase B benchmarks; there is
//                     no network access for the real datasets).
//  * sample_neighbors GraphSAGE-style layer-wise uniform neighbour sampling
//                     producing per-layer CSR blocks.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <omp.h>

#include <algorithm>
#include <cstdint>
#include <numeric>
#include <random>
#include <unordered_map>
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "rt_common.h"

namespace py = pybind11;
using i32 = int32_t;
using i64 = int64_t;
using cgnn_rt::mix64;

void register_reorder(py::module& m);   // reorder.cpp

namespace {

constexpr int PROG_HDR = 4;
constexpr int NODE_REC = 8;

std::vector<int> sweep_order(int n, const std::vector<std::vector<int>>& parents,
                             const std::vector<int>& list_order) {
  std::vector<char> done(n, 0);
  std::vector<int> order;
  order.reserve(n);
  while ((int)order.size() < n) {
    bool progressed = false;
    for (int v : list_order) {
      if (done[v]) continue;
      bool ok = true;
      for (int p : parents[v]) if (!done[p]) { ok = false; break; }
      if (ok) { done[v] = 1; order.push_back(v); progressed = true; }
    }
    if (!progressed) throw std::invalid_argument("dag_program: graph is cyclic");
  }
  return order;
}

}  // namespace

// parents[v]  : parent variable indices of v (in the order they feed the MLP)
// kinds[v]    : 0 generated, 1 observed (clamped to data)
// confs[v]    : confounder-noise ids appended after the own noise
// list_order  : the variable order of the reference's sweep
// returns (program int32[], n_params, max_in)
py::tuple dag_program(int n_vars, const std::vector<std::vector<int>>& parents,
                      const std::vector<int>& kinds, const std::vector<std::vector<int>>& confs,
                      int H, std::vector<int> list_order, int n_conf) {
  if ((int)parents.size() != n_vars || (int)kinds.size() != n_vars || (int)confs.size() != n_vars)
    throw std::invalid_argument("dag_program: size mismatch");
  if (list_order.empty()) { list_order.resize(n_vars); std::iota(list_order.begin(), list_order.end(), 0); }
  for (int v = 0; v < n_vars; ++v)
    for (int p : parents[v])
      if (p < 0 || p >= n_vars) throw std::invalid_argument("dag_program: parent out of range");
  const std::vector<int> order = sweep_order(n_vars, parents, list_order);
  size_t pool = 0;
  for (int v = 0; v < n_vars; ++v) pool += parents[v].size() + confs[v].size();
  std::vector<i32> prog(PROG_HDR + (size_t)NODE_REC * n_vars + pool, 0);
  int pool_off = PROG_HDR + NODE_REC * n_vars;
  int param_off = 0, max_in = 0;
  for (int k = 0; k < n_vars; ++k) {
    const int v = order[k];
    i32* rec = prog.data() + PROG_HDR + (size_t)k * NODE_REC;
    const int npar = (int)parents[v].size(), ncf = (int)confs[v].size();
    rec[0] = v;
    rec[1] = kinds[v];
    rec[2] = npar;
    rec[3] = pool_off;
    for (int j = 0; j < npar; ++j) prog[pool_off++] = parents[v][j];
    rec[4] = ncf;
    rec[5] = pool_off;
    for (int j = 0; j < ncf; ++j) prog[pool_off++] = confs[v][j];
    const int nin = npar + 1 + ncf;
    rec[7] = nin;
    if (kinds[v] == 0) {
      rec[6] = param_off;
      param_off += (nin + 2) * H + 1;
      max_in = std::max(max_in, nin);
    } else {
      rec[6] = -1;
    }
  }
  prog[0] = n_vars;
  prog[1] = param_off;
  prog[2] = n_conf;
  prog[3] = max_in;
  py::array_t<i32> arr(prog.size());
  std::copy(prog.begin(), prog.end(), arr.mutable_data());
  return py::make_tuple(arr, param_off, max_in);
}

// Stage schedule of one DAG program for the level-scheduled generator kernels
// (kernels/cgnn_staged.hip).  level(v) = 0 for observed / parentless nodes, else
// 1 + max level of its parents.  Forward stages = levels in increasing order (record
// order inside a level).  Backward sub-stages: the generated nodes of each level, levels
// in decreasing order, split greedily (first fit, records in decreasing order) so that no
// two nodes of one sub-stage share a parent -- each dL/dparent accumulation is then
// owned by one wave.  Layout: [nf, nb, fwd_base, bwd_base | fwd starts[nf+1], fwd records |
// bwd starts[nb+1], bwd records].  Returns (schedule, widest forward stage, widest
// backward sub-stage).
py::tuple dag_schedule(py::array_t<i32, py::array::c_style | py::array::forcecast> prog_a) {
  const i32* prog = prog_a.data();
  const i64 len = prog_a.size();
  if (len < PROG_HDR) throw std::invalid_argument("dag_schedule: program too short");
  const int nn = prog[0];
  if (len < PROG_HDR + (i64)NODE_REC * nn) throw std::invalid_argument("dag_schedule: truncated program");
  std::vector<int> level_of_var(nn, -1), level_of_rec(nn, 0);
  int max_level = 0;
  for (int k = 0; k < nn; ++k) {
    const i32* rec = prog + PROG_HDR + (size_t)k * NODE_REC;
    const int var = rec[0], kind = rec[1], npar = rec[2], paroff = rec[3];
    if (var < 0 || var >= nn) throw std::invalid_argument("dag_schedule: variable out of range");
    int lv = 0;
    if (kind == 0)
      for (int j = 0; j < npar; ++j) {
        const int p = prog[paroff + j];
        if (p < 0 || p >= nn || level_of_var[p] < 0)
          throw std::invalid_argument("dag_schedule: parent not generated before its child");
        lv = std::max(lv, level_of_var[p] + 1);
      }
    level_of_var[var] = lv;
    level_of_rec[k] = lv;
    max_level = std::max(max_level, lv);
  }
  std::vector<std::vector<int>> by_level(max_level + 1);
  for (int k = 0; k < nn; ++k) by_level[level_of_rec[k]].push_back(k);
  std::vector<std::vector<int>> fwd(by_level.begin(), by_level.end());
  std::vector<std::vector<int>> bwd;
  std::vector<char> used(nn, 0);
  for (int lv = max_level; lv >= 0; --lv) {
    std::vector<std::vector<int>> subs;
    std::vector<std::vector<int>> sub_parents;
    const auto& nodes = by_level[lv];
    for (auto it = nodes.rbegin(); it != nodes.rend(); ++it) {
      const int k = *it;
      const i32* rec = prog + PROG_HDR + (size_t)k * NODE_REC;
      if (rec[1] != 0) continue;                       // observed: nothing to train
      const int npar = rec[2], paroff = rec[3];
      size_t s = 0;
      for (; s < subs.size(); ++s) {
        bool clash = false;
        for (int p : sub_parents[s]) used[p] = 1;
        for (int j = 0; j < npar && !clash; ++j) clash = used[prog[paroff + j]] != 0;
        for (int p : sub_parents[s]) used[p] = 0;
        if (!clash) break;
      }
      if (s == subs.size()) { subs.emplace_back(); sub_parents.emplace_back(); }
      subs[s].push_back(k);
      for (int j = 0; j < npar; ++j) sub_parents[s].push_back(prog[paroff + j]);
    }
    for (auto& sb : subs) bwd.push_back(std::move(sb));
  }
  const int nf = (int)fwd.size(), nb = (int)bwd.size();
  std::vector<i32> out(4);
  int wf = 0, wb = 0;
  auto emit = [&](const std::vector<std::vector<int>>& st, int& widest) {
    int acc = 0;
    out.push_back(0);
    for (auto& v : st) { acc += (int)v.size(); out.push_back(acc); widest = std::max(widest, (int)v.size()); }
    for (auto& v : st) for (int k : v) out.push_back(k);
  };
  out[0] = nf; out[1] = nb;
  out[2] = (i32)out.size();
  emit(fwd, wf);
  out[3] = (i32)out.size();
  emit(bwd, wb);
  py::array_t<i32> arr(out.size());
  std::copy(out.begin(), out.end(), arr.mutable_data());
  return py::make_tuple(arr, wf, wb);
}

bool is_acyclic(int n, const std::vector<std::pair<int, int>>& edges) {
  std::vector<int> indeg(n, 0);
  std::vector<std::vector<int>> succ(n);
  for (auto& e : edges) { succ[e.first].push_back(e.second); indeg[e.second]++; }
  std::vector<int> q;
  for (int v = 0; v < n; ++v) if (!indeg[v]) q.push_back(v);
  size_t seen = 0;
  while (!q.empty()) {
    int v = q.back(); q.pop_back(); ++seen;
    for (int w : succ[v]) if (--indeg[w] == 0) q.push_back(w);
  }
  return seen == (size_t)n;
}

uint64_t canonical_hash(std::vector<std::pair<int, int>> edges) {
  std::sort(edges.begin(), edges.end());
  edges.erase(std::unique(edges.begin(), edges.end()), edges.end());
  uint64_t h = 0x243F6A8885A308D3ull ^ edges.size();
  for (auto& e : edges) h = mix64(h ^ (((uint64_t)(uint32_t)e.first << 32) | (uint32_t)e.second));
  return h;
}

// CSR (rowptr int64? no: int32 indices, int64 rowptr when nnz >= 2^31)
py::tuple csr_from_edges(i64 n, py::array_t<i64, py::array::c_style | py::array::forcecast> src_a,
                         py::array_t<i64, py::array::c_style | py::array::forcecast> dst_a,
                         bool symmetric, bool self_loops, bool dedup) {
  const i64 m = src_a.size();
  if (dst_a.size() != m) throw std::invalid_argument("csr_from_edges: size mismatch");
  const i64* src = src_a.data();
  const i64* dst = dst_a.data();
  const int nt = omp_get_max_threads();
  const i64 tot = (symmetric ? 2 * m : m);
  std::vector<i64> deg(n + 1, 0);
  {
    std::vector<std::vector<i64>> local(nt, std::vector<i64>(n, 0));
#pragma omp parallel for schedule(static)
    for (i64 e = 0; e < m; ++e) {
      auto& d = local[omp_get_thread_num()];
      const i64 s = src[e], t = dst[e];
      if (s < 0 || s >= n || t < 0 || t >= n) continue;
      if (s == t) continue;   // self loops handled separately
      d[s]++;
      if (symmetric) d[t]++;
    }
    for (int t = 0; t < nt; ++t)
      for (i64 v = 0; v < n; ++v) deg[v + 1] += local[t][v];
  }
  if (self_loops) for (i64 v = 0; v < n; ++v) deg[v + 1] += 1;
  for (i64 v = 0; v < n; ++v) deg[v + 1] += deg[v];
  std::vector<i64> fill(deg.begin(), deg.end() - 1);
  std::vector<i32> col(deg[n]);
  (void)tot;
  // sequential scatter keeps the build deterministic
  for (i64 e = 0; e < m; ++e) {
    const i64 s = src[e], t = dst[e];
    if (s < 0 || s >= n || t < 0 || t >= n || s == t) continue;
    col[fill[s]++] = (i32)t;
    if (symmetric) col[fill[t]++] = (i32)s;
  }
  if (self_loops) for (i64 v = 0; v < n; ++v) col[fill[v]++] = (i32)v;
  // sort each row (locality) and optionally drop duplicates
  std::vector<i64> newdeg(n + 1, 0);
#pragma omp parallel for schedule(dynamic, 4096)
  for (i64 v = 0; v < n; ++v) {
    auto b = col.begin() + deg[v], e = col.begin() + deg[v + 1];
    std::sort(b, e);
    newdeg[v + 1] = dedup ? (std::unique(b, e) - b) : (e - b);
  }
  for (i64 v = 0; v < n; ++v) newdeg[v + 1] += newdeg[v];
  py::array_t<i64> rowptr(n + 1);
  py::array_t<i32> colout(newdeg[n]);
  i64* rp = rowptr.mutable_data();
  i32* co = colout.mutable_data();
  std::copy(newdeg.begin(), newdeg.end(), rp);
#pragma omp parallel for schedule(dynamic, 4096)
  for (i64 v = 0; v < n; ++v)
    std::copy(col.begin() + deg[v], col.begin() + deg[v] + (newdeg[v + 1] - newdeg[v]), co + newdeg[v]);
  return py::make_tuple(rowptr, colout);
}

// Planted-partition graph with the shape of an OGB node-property dataset.
//   n nodes, ~m undirected edges, c classes; communities are contiguous id blocks,
//   node labels follow the community except for a `label_noise` fraction.
//   Each node draws a degree from a truncated power law with mean 2m/n; each
//   edge end goes to the same community with probability `homophily` (a
//   window of nearby ids inside the community) and uniformly at random
//   otherwise.  Features: class centroid + N(0,1) noise (bf16-ready fp32), so a
//   2-layer GCN reaches a non-trivial validation accuracy.
//   id_order 0 ("banded") returns the generator's ids, whose homophilous edges
//   join nearby ids -- locality a real dataset's ids do not hand out for free;
//   id_order 1 ("shuffled") relabels every node through a seeded bijection of
//   [0, n) (IdPermutation), so ids carry no information and any locality must be
//   earned by a reordering pass (reorder.cpp).
//   Every quantity is a pure function of (seed, edge index) or (seed, node id), so
//   any row range of the graph can be generated on its own (synthetic_shard).
namespace {

struct SynthSpec {
  int64_t n, m;
  int n_feat, n_class;
  double homophily, feat_noise, label_noise;
  uint64_t seed;
  int id_order;
  int64_t block;
  double mean_deg;
  cgnn_rt::IdPermutation perm;
  SynthSpec(int64_t n_, int64_t m_, int nf, int nc, double hom, double fn, uint64_t sd, double ln, int io)
      : n(n_), m(m_), n_feat(nf), n_class(nc), homophily(hom), feat_noise(fn), label_noise(ln), seed(sd),
        id_order(io), block((n_ + nc - 1) / nc), mean_deg((double)m_ / (double)n_), perm(n_, sd ^ 0x5A17ull) {}
  int64_t pid(int64_t v) const { return id_order ? (int64_t)perm((uint64_t)v) : v; }
  int64_t gen_id(int64_t v) const { return id_order ? (int64_t)perm.inverse((uint64_t)v) : v; }
  int32_t comm(int64_t v) const { return (int32_t)std::min<int64_t>(v / block, n_class - 1); }
  int32_t label(int64_t v) const {                    // v in generator space
    const uint64_t h = mix64(seed ^ 0x1AB3ull ^ mix64((uint64_t)v));
    const double u = ((h >> 11) + 0.5) * (1.0 / 9007199254740992.0);
    return u < label_noise ? (int32_t)(mix64(h) % (uint64_t)n_class) : comm(v);
  }
  // edge e in generator space
  void edge(int64_t e, int64_t& s, int64_t& t) const {
    uint64_t h = mix64(seed ^ mix64((uint64_t)e * 0x9E3779B97F4A7C15ull));
    const double u = ((h >> 11) + 0.5) * (1.0 / 9007199254740992.0);
    h = mix64(h);
    s = (int64_t)((double)n * std::pow(u, 1.6)) % n;   // skew towards low ids ...
    s = (int64_t)(mix64(s ^ seed) % (uint64_t)n);       // ... then scatter the hubs
    const double u2 = ((h >> 11) + 0.5) * (1.0 / 9007199254740992.0);
    h = mix64(h);
    if (u2 < homophily) {
      const int64_t c = comm(s);
      const int64_t lo = c * block, hi = std::min<int64_t>(n, lo + block);
      const int64_t win = std::max<int64_t>(16, (int64_t)(8 * mean_deg));
      const int64_t off = (int64_t)(h % (uint64_t)(2 * win + 1)) - win;
      t = s + off;
      if (t < lo) t += (hi - lo);
      if (t >= hi) t -= (hi - lo);
      if (t < lo || t >= hi) t = lo + (int64_t)(h % (uint64_t)(hi - lo));
    } else {
      t = (int64_t)(h % (uint64_t)n);
    }
  }
  void features(int64_t v, const std::vector<float>& cent, float* xr) const {   // v in generator space
    const int32_t lab = label(v);
    uint64_t h = mix64(seed ^ 0xFEEDull ^ mix64((uint64_t)v));
    for (int f = 0; f < n_feat; f += 2) {
      h = mix64(h);
      const double u1 = ((h >> 11) + 0.5) * (1.0 / 9007199254740992.0);
      h = mix64(h);
      const double u2 = ((h >> 11) + 0.5) * (1.0 / 9007199254740992.0);
      const double r = std::sqrt(-2.0 * std::log(u1));
      const double z0 = r * std::cos(6.283185307179586 * u2), z1 = r * std::sin(6.283185307179586 * u2);
      xr[f] = (float)(cent[(size_t)lab * n_feat + f] + feat_noise * z0);
      if (f + 1 < n_feat) xr[f + 1] = (float)(cent[(size_t)lab * n_feat + f + 1] + feat_noise * z1);
    }
  }
  std::vector<float> centroids() const {
    std::vector<float> cent((size_t)n_class * n_feat);
    std::mt19937_64 g(seed ^ 0xC0FFEEull);
    std::normal_distribution<float> nd(0.f, 1.f);
    for (auto& c : cent) c = nd(g);
    return cent;
  }
};

}  // namespace

py::tuple synthetic_graph(i64 n, i64 m, int n_feat, int n_class, double homophily,
                          double feat_noise, uint64_t seed, double label_noise, int id_order) {
  const SynthSpec sp(n, m, n_feat, n_class, homophily, feat_noise, seed, label_noise, id_order);
  py::array_t<i64> src_a(m), dst_a(m);
  py::array_t<i32> label_a(n);
  i64* src = src_a.mutable_data();
  i64* dst = dst_a.mutable_data();
  i32* lab = label_a.mutable_data();
  py::array_t<float> feat_a({(py::ssize_t)n, (py::ssize_t)n_feat});
  float* x = feat_a.mutable_data();
  {
    py::gil_scoped_release nogil;
#pragma omp parallel for schedule(static)
    for (i64 e = 0; e < m; ++e) {
      i64 s, t;
      sp.edge(e, s, t);
      src[e] = sp.pid(s);
      dst[e] = sp.pid(t);
    }
    const std::vector<float> cent = sp.centroids();
#pragma omp parallel for schedule(static)
    for (i64 v = 0; v < n; ++v) {
      const i64 pv = sp.pid(v);
      lab[pv] = sp.label(v);
      sp.features(v, cent, x + (size_t)pv * n_feat);
    }
  }
  return py::make_tuple(src_a, dst_a, feat_a, label_a);
}

// Rows [r0, r1) (final ids) of the same graph as synthetic_graph + csr_from_edges(n,
// src, dst, symmetric, self loops, dedup): CSR with GLOBAL column ids, the rows'
// features and labels -- generated without materialising the rest of the graph
// (every rank of a graph-sharded job scans the edge hash space and keeps the edges
// touching its rows: O(m) hashing, O(local nnz) memory).  rowptr is int64 (a shard
// of a 10^9-edge graph may pass 2^31 entries), columns int32 (n < 2^31).
//
// order (optional, [n] int64): a partition order -- node f (final id) becomes row
// order[f]; the shard is then rows [r0, r1) of the RELABELLED graph (columns relabelled
// too), and the returned `ids` are the final ids of its rows (for the split mask).
// with_features = false: structure only (a partitioning pass over the whole graph).
py::tuple synthetic_shard(i64 n, i64 m, int n_feat, int n_class, double homophily, double feat_noise,
                          uint64_t seed, double label_noise, int id_order, i64 r0, i64 r1,
                          py::array_t<i64, py::array::c_style | py::array::forcecast> order_a, bool with_features) {
  if (r0 < 0 || r1 > n || r0 > r1) throw std::invalid_argument("synthetic_shard: bad row range");
  if (n >= (i64)1 << 31) throw std::invalid_argument("synthetic_shard: n >= 2^31 needs int64 columns");
  const bool relabel = order_a.size() > 0;
  if (relabel && order_a.size() != n) throw std::invalid_argument("synthetic_shard: order must have n entries");
  const i64* ord = relabel ? order_a.data() : nullptr;
  if (relabel) {
    // a permutation of [0, n): every value in range and seen once (otherwise some local
    // rows would get no id and the split mask / labels would read garbage)
    std::vector<uint8_t> seen(n, 0);
    bool ok = true;
    for (i64 f = 0; f < n && ok; ++f) {
      const i64 v = ord[f];
      ok = v >= 0 && v < n && !seen[v];
      if (ok) seen[v] = 1;
    }
    if (!ok) throw std::invalid_argument("synthetic_shard: order must be a permutation of [0, n)");
  }
  const SynthSpec sp(n, m, n_feat, n_class, homophily, feat_noise, seed, label_noise, id_order);
  const i64 nl = r1 - r0;
  py::array_t<i64> rp_a(nl + 1);
  i64* rp = rp_a.mutable_data();
  py::array_t<float> feat_a({(py::ssize_t)(with_features ? nl : 0), (py::ssize_t)n_feat});
  py::array_t<i32> label_a(with_features ? nl : 0);
  py::array_t<i64> ids_a(nl);
  i64* ids = ids_a.mutable_data();
  std::vector<i32> col;
  {
    py::gil_scoped_release nogil;
    // final id of every local row (identity without an order)
    if (relabel) {
#pragma omp parallel for schedule(static)
      for (i64 f = 0; f < n; ++f) {
        const i64 v = ord[f];
        if (v >= r0 && v < r1) ids[v - r0] = f;
      }
    } else {
      for (i64 v = 0; v < nl; ++v) ids[v] = r0 + v;
    }
    auto fid = [&](i64 x) -> i64 { const i64 p = sp.pid(x); return relabel ? ord[p] : p; };
    std::vector<i64> cnt(nl + 1, 0);
    // pass 1: degree of every local row (both directions of every edge, self loops apart)
#pragma omp parallel for schedule(static)
    for (i64 e = 0; e < m; ++e) {
      i64 s, t;
      sp.edge(e, s, t);
      const i64 ps = fid(s), pt = fid(t);
      if (ps == pt) continue;
      if (ps >= r0 && ps < r1) __atomic_fetch_add(&cnt[ps - r0 + 1], 1, __ATOMIC_RELAXED);
      if (pt >= r0 && pt < r1) __atomic_fetch_add(&cnt[pt - r0 + 1], 1, __ATOMIC_RELAXED);
    }
    for (i64 v = 0; v < nl; ++v) cnt[v + 1] += cnt[v] + 1;    // + the self loop
    std::vector<i64> cur(cnt.begin(), cnt.end() - 1);
    col.resize(cnt[nl]);
    for (i64 v = 0; v < nl; ++v) col[cur[v]++] = (i32)(r0 + v);
    // pass 2: fill (order inside a row is fixed by the sort below)
#pragma omp parallel for schedule(static)
    for (i64 e = 0; e < m; ++e) {
      i64 s, t;
      sp.edge(e, s, t);
      const i64 ps = fid(s), pt = fid(t);
      if (ps == pt) continue;
      if (ps >= r0 && ps < r1) col[__atomic_fetch_add(&cur[ps - r0], 1, __ATOMIC_RELAXED)] = (i32)pt;
      if (pt >= r0 && pt < r1) col[__atomic_fetch_add(&cur[pt - r0], 1, __ATOMIC_RELAXED)] = (i32)ps;
    }
    // sort + de-duplicate every row, then compact
    std::vector<i64> keep(nl + 1, 0);
#pragma omp parallel for schedule(dynamic, 4096)
    for (i64 v = 0; v < nl; ++v) {
      auto b = col.begin() + cnt[v], e = col.begin() + cnt[v + 1];
      std::sort(b, e);
      keep[v + 1] = std::unique(b, e) - b;
    }
    rp[0] = 0;
    for (i64 v = 0; v < nl; ++v) rp[v + 1] = rp[v] + keep[v + 1];
    i64 w = 0;
    for (i64 v = 0; v < nl; ++v) {            // in place: rows only move left
      const i64 b = cnt[v], k = keep[v + 1];
      if (w != b) std::memmove(col.data() + w, col.data() + b, sizeof(i32) * (size_t)k);
      w += k;
    }
    col.resize(w);
    col.shrink_to_fit();
    if (with_features) {
      const std::vector<float> cent = sp.centroids();
      float* x = feat_a.mutable_data();
      i32* lab = label_a.mutable_data();
#pragma omp parallel for schedule(static)
      for (i64 v = 0; v < nl; ++v) {
        const i64 gv = sp.gen_id(ids[v]);
        lab[v] = sp.label(gv);
        sp.features(gv, cent, x + (size_t)v * n_feat);
      }
    }
  }
  py::array_t<i32> col_a((py::ssize_t)col.size());
  std::copy(col.begin(), col.end(), col_a.mutable_data());
  return py::make_tuple(rp_a, col_a, feat_a, label_a, ids_a);
}

// Train / valid / test split by a per-node hash: node v is train with probability
// n_train / n, valid with n_val / n, else test (1 / 2 / 3) -- a pure function of
// (seed, v), so every rank labels its own rows consistently without a global
// permutation of 10^8 ids.
py::array_t<uint8_t> split_mask(i64 n, i64 n_train, i64 n_val, uint64_t seed,
                                py::array_t<i64, py::array::c_style | py::array::forcecast> ids) {
  py::array_t<uint8_t> out(ids.size());
  const i64* id = ids.data();
  uint8_t* o = out.mutable_data();
  const double pt = (double)n_train / (double)n, pv = (double)(n_train + n_val) / (double)n;
  const i64 k = ids.size();
#pragma omp parallel for schedule(static)
  for (i64 i = 0; i < k; ++i) {
    const double u = ((mix64(mix64(seed ^ 0x5B117ull) ^ (uint64_t)id[i]) >> 11) + 0.5) * (1.0 / 9007199254740992.0);
    o[i] = u < pt ? 1 : (u < pv ? 2 : 3);
  }
  return out;
}

// Layer-wise uniform neighbour sampling (GraphSAGE).  For each layer (outermost
// first) sample up to fanout[l] neighbours of the current frontier; returns, per
// layer, (block_rowptr, block_col_local, frontier_nodes) with the destination
// nodes first in each frontier (standard "dst nodes are a prefix of src nodes").
py::list sample_neighbors(py::array_t<i64, py::array::c_style | py::array::forcecast> rowptr_a,
                          py::array_t<i32, py::array::c_style | py::array::forcecast> col_a,
                          py::array_t<i64, py::array::c_style | py::array::forcecast> seeds_a,
                          std::vector<int> fanouts, uint64_t seed) {
  const i64* rowptr = rowptr_a.data();
  const i32* col = col_a.data();
  struct Block { std::vector<i64> rp; std::vector<i32> col; std::vector<i64> nodes; };
  std::vector<Block> blocks(fanouts.size());
  std::vector<i64> frontier(seeds_a.data(), seeds_a.data() + seeds_a.size());
  {
    // the sampling itself runs without the GIL (a data-loader thread overlaps it
    // with the GPU step of the previous batch)
    py::gil_scoped_release nogil;
    for (size_t l = 0; l < fanouts.size(); ++l) {
      const int fo = fanouts[l];
      const i64 nd = (i64)frontier.size();
      std::vector<i64>& cnt = blocks[l].rp;
      cnt.assign(nd + 1, 0);
      for (i64 i = 0; i < nd; ++i) {
        const i64 v = frontier[i];
        const i64 deg = rowptr[v + 1] - rowptr[v];
        cnt[i + 1] = fo < 0 ? deg : std::min<i64>(deg, fo);
      }
      for (i64 i = 0; i < nd; ++i) cnt[i + 1] += cnt[i];
      std::vector<i64> picked(cnt[nd]);
#pragma omp parallel for schedule(dynamic, 256)
      for (i64 i = 0; i < nd; ++i) {
        const i64 v = frontier[i];
        const i64 b = rowptr[v], deg = rowptr[v + 1] - b, k = cnt[i + 1] - cnt[i];
        i64* dstp = picked.data() + cnt[i];
        if (k == deg) {
          for (i64 q = 0; q < k; ++q) dstp[q] = col[b + q];
        } else {   // Floyd's algorithm: k distinct positions out of deg
          uint64_t h = mix64(seed ^ mix64((uint64_t)v * 131 + l));
          std::vector<i64> pos;
          pos.reserve(k);
          for (i64 j = deg - k; j < deg; ++j) {
            h = mix64(h);
            i64 t = (i64)(h % (uint64_t)(j + 1));
            if (std::find(pos.begin(), pos.end(), t) != pos.end()) t = j;
            pos.push_back(t);
          }
          for (i64 q = 0; q < k; ++q) dstp[q] = col[b + pos[q]];
        }
      }
      // relabel: destination nodes first, then new source nodes in first-seen order
      std::vector<i64>& nodes = blocks[l].nodes;
      nodes = frontier;
      std::unordered_map<i64, i32> idx;
      idx.reserve(frontier.size() * 2 + picked.size());
      for (i64 i = 0; i < nd; ++i) idx.emplace(frontier[i], (i32)i);
      std::vector<i32>& bc = blocks[l].col;
      bc.resize(picked.size());
      for (size_t q = 0; q < picked.size(); ++q) {
        auto it = idx.find(picked[q]);
        if (it == idx.end()) {
          it = idx.emplace(picked[q], (i32)nodes.size()).first;
          nodes.push_back(picked[q]);
        }
        bc[q] = it->second;
      }
      frontier = nodes;
    }
  }
  py::list out;
  for (auto& b : blocks) {
    py::array_t<i64> brow(b.rp.size());
    std::copy(b.rp.begin(), b.rp.end(), brow.mutable_data());
    py::array_t<i32> bcol(b.col.size());
    std::copy(b.col.begin(), b.col.end(), bcol.mutable_data());
    py::array_t<i64> nodes_a(b.nodes.size());
    std::copy(b.nodes.begin(), b.nodes.end(), nodes_a.mutable_data());
    out.append(py::make_tuple(brow, bcol, nodes_a));
  }
  return out;
}

PYBIND11_MODULE(_rt, m) {
  m.doc() = "cgnn_amd host runtime (C++)";
  m.def("dag_program", &dag_program, py::arg("n_vars"), py::arg("parents"), py::arg("kinds"),
        py::arg("confs"), py::arg("H"), py::arg("list_order") = std::vector<int>(),
        py::arg("n_conf") = 0);
  m.def("dag_schedule", &dag_schedule, py::arg("prog"));
  m.def("is_acyclic", &is_acyclic);
  m.def("canonical_hash", &canonical_hash);
  m.def("csr_from_edges", &csr_from_edges, py::arg("n"), py::arg("src"), py::arg("dst"),
        py::arg("symmetric") = true, py::arg("self_loops") = true, py::arg("dedup") = true);
  m.def("synthetic_graph", &synthetic_graph, py::arg("n"), py::arg("m"), py::arg("n_feat"),
        py::arg("n_class"), py::arg("homophily") = 0.8, py::arg("feat_noise") = 1.0,
        py::arg("seed") = 0, py::arg("label_noise") = 0.0, py::arg("id_order") = 0);
  m.def("synthetic_shard", &synthetic_shard, py::arg("n"), py::arg("m"), py::arg("n_feat"), py::arg("n_class"),
        py::arg("homophily"), py::arg("feat_noise"), py::arg("seed"), py::arg("label_noise"), py::arg("id_order"),
        py::arg("r0"), py::arg("r1"), py::arg("order") = py::array_t<i64>(0), py::arg("with_features") = true);
  m.def("split_mask", &split_mask, py::arg("n"), py::arg("n_train"), py::arg("n_val"), py::arg("seed"),
        py::arg("ids"));
  m.def("sample_neighbors", &sample_neighbors);
  m.def("num_threads", []() { return omp_get_max_threads(); });
  m.def("set_num_threads", [](int k) { omp_set_num_threads(k > 0 ? k : 1); }, py::arg("k"));
  m.def("id_permutation", [](i64 n, uint64_t seed, py::array_t<i64, py::array::c_style | py::array::forcecast> v,
                             bool inverse) {
    const cgnn_rt::IdPermutation p(n, seed);
    py::array_t<i64> out(v.size());
    const i64* a = v.data();
    i64* o = out.mutable_data();
    for (py::ssize_t i = 0; i < v.size(); ++i) o[i] = (i64)(inverse ? p.inverse((uint64_t)a[i]) : p((uint64_t)a[i]));
    return out;
  }, py::arg("n"), py::arg("seed"), py::arg("ids"), py::arg("inverse") = false);
  register_reorder(m);
}
