// Locality reordering of node ids (GNN track, not in the reference).
//
// The gathers of a CSR SpMM read the feature row of every neighbour; when the
// neighbours of consecutive rows have nearby ids those rows are reused from L2
// and the Infinity Cache instead of HBM.  Real graph ids carry no such order (and
// the synthetic generator scrambles its ids by default), so the framework earns
// the locality itself with a reordering pass run once at setup:
//
//   1. clustering by size-capped label propagation: every node repeatedly adopts
//      the label most frequent among its neighbours; updates alternate between two
//      hash-selected halves of the nodes reading a snapshot (deterministic for any
//      thread count, and no two-colour oscillation); a label that already holds
//      `max_cluster` nodes accepts no new members, so clusters stay cache-sized;
//   2. cluster order: clusters are laid out by a depth-first walk of the cluster
//      graph (strongest link first), so clusters joined by many edges sit next to
//      each other;
//   3. inside a cluster: Cuthill-McKee (BFS from a minimum-degree node, neighbours
//      in ascending degree) over the intra-cluster edges, which lines up band /
//      chain structure so that consecutive rows share most of their neighbours;
//   4. refinement (`locality_refine`): a few rounds of median smoothing of the
//      positions, which narrows the band across cluster boundaries (products shape:
//      edges within +-256 positions 56 % -> 74 % after 4 rounds, within +-128
//      34 % -> 50 %).
//
// Everything is O(nnz log deg) and OpenMP-parallel; the result is a permutation
// `new_id[old]`.  `locality_stats` measures an order: the fraction of edges whose
// endpoints are within w positions of each other for a few windows w (the reuse a
// row-ordered gather kernel can see from L2 / the Infinity Cache).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <omp.h>

#include <algorithm>
#include <cstdint>
#include <numeric>
#include <stdexcept>
#include <utility>
#include <vector>

#include "rt_common.h"

namespace py = pybind11;
using i32 = int32_t;
using i64 = int64_t;
using cgnn_rt::mix64;

namespace {

using I64Arr = py::array_t<i64, py::array::c_style | py::array::forcecast>;
using I32Arr = py::array_t<i32, py::array::c_style | py::array::forcecast>;

// size-capped, half-synchronous label propagation; returns labels in [0, n)
std::vector<i64> label_propagation(i64 n, const i64* rp, const i32* col, int rounds, i64 cap,
                                   uint64_t seed) {
  std::vector<i64> lab(n), nxt(n), size(n, 1);
  std::iota(lab.begin(), lab.end(), 0);
  const int nt = omp_get_max_threads();
  std::vector<std::vector<i64>> bufs(nt);
  for (int r = 0; r < rounds; ++r) {
    for (int phase = 0; phase < 2; ++phase) {
      i64 changed = 0;
#pragma omp parallel for schedule(dynamic, 2048) reduction(+ : changed)
      for (i64 v = 0; v < n; ++v) {
        nxt[v] = lab[v];
        if ((i64)(mix64(seed ^ (uint64_t)v ^ ((uint64_t)r << 40)) & 1) != phase) continue;
        auto& buf = bufs[omp_get_thread_num()];
        buf.clear();
        for (i64 e = rp[v]; e < rp[v + 1]; ++e)
          if (col[e] != v) buf.push_back(lab[col[e]]);
        if (buf.empty()) continue;
        std::sort(buf.begin(), buf.end());
        const i64 cur = lab[v];
        i64 best = cur, best_cnt = 0, cur_cnt = 0;
        for (size_t i = 0; i < buf.size();) {
          size_t j = i;
          while (j < buf.size() && buf[j] == buf[i]) ++j;
          const i64 l = buf[i], c = (i64)(j - i);
          if (l == cur) cur_cnt = c;
          else if (c > best_cnt && size[l] < cap) { best = l; best_cnt = c; }
          i = j;
        }
        if (best_cnt > cur_cnt) { nxt[v] = best; ++changed; }
      }
      std::swap(lab, nxt);
      std::fill(size.begin(), size.end(), 0);
#pragma omp parallel for schedule(static)
      for (i64 v = 0; v < n; ++v) {
#pragma omp atomic
        size[lab[v]] += 1;
      }
      if (changed == 0 && phase == 1) return lab;
    }
  }
  return lab;
}

}  // namespace

// Locality-improving node order.  Returns new_id[old] (int64).
py::array_t<i64> locality_order(i64 n, I64Arr rowptr_a, I32Arr col_a, int lp_rounds, i64 max_cluster,
                                uint64_t seed) {
  if (rowptr_a.size() != n + 1) throw std::invalid_argument("locality_order: rowptr size");
  const i64* rp = rowptr_a.data();
  const i32* col = col_a.data();
  if (rp[n] != (i64)col_a.size()) throw std::invalid_argument("locality_order: col size");
  py::array_t<i64> out(n);
  i64* new_id = out.mutable_data();
  {
    py::gil_scoped_release nogil;
    const std::vector<i64> lab = label_propagation(n, rp, col, lp_rounds, std::max<i64>(max_cluster, 1), seed);
    // clusters: counting sort of the nodes by label
    std::vector<i64> coff(n + 1, 0);
    for (i64 v = 0; v < n; ++v) coff[lab[v] + 1]++;
    for (i64 l = 0; l < n; ++l) coff[l + 1] += coff[l];
    std::vector<i64> members(n);
    {
      std::vector<i64> fill(coff.begin(), coff.end() - 1);
      for (i64 v = 0; v < n; ++v) members[fill[lab[v]]++] = v;
    }
    std::vector<i64> cl_ids;                 // non-empty labels
    for (i64 l = 0; l < n; ++l) if (coff[l + 1] > coff[l]) cl_ids.push_back(l);
    const i64 ncl = (i64)cl_ids.size();
    std::vector<i64> cl_index(n, -1);
    for (i64 k = 0; k < ncl; ++k) cl_index[cl_ids[k]] = k;
    // cluster graph: for every cluster the other clusters it links to, by edge count
    std::vector<std::vector<std::pair<i64, i64>>> cadj(ncl);   // (count, neighbour cluster)
#pragma omp parallel for schedule(dynamic, 64)
    for (i64 k = 0; k < ncl; ++k) {
      const i64 l = cl_ids[k];
      std::vector<i64> nb;
      for (i64 q = coff[l]; q < coff[l + 1]; ++q) {
        const i64 v = members[q];
        for (i64 e = rp[v]; e < rp[v + 1]; ++e) {
          const i64 lu = lab[col[e]];
          if (lu != l) nb.push_back(cl_index[lu]);
        }
      }
      std::sort(nb.begin(), nb.end());
      auto& out_k = cadj[k];
      for (size_t i = 0; i < nb.size();) {
        size_t j = i;
        while (j < nb.size() && nb[j] == nb[i]) ++j;
        out_k.emplace_back((i64)(j - i), nb[i]);
        i = j;
      }
      std::sort(out_k.begin(), out_k.end(), [](const std::pair<i64, i64>& a, const std::pair<i64, i64>& b) {
        return a.first != b.first ? a.first > b.first : a.second < b.second;
      });
    }
    // cluster order: depth-first walk of the cluster graph, strongest link first (the next
    // cluster is the most strongly linked unplaced neighbour of the last one, so chains of
    // clusters -- e.g. consecutive segments of a band -- are laid out in sequence); restarts
    // from the largest unplaced cluster
    std::vector<i64> corder;
    corder.reserve(ncl);
    {
      std::vector<char> placed(ncl, 0);
      std::vector<i64> by_size(ncl);
      std::iota(by_size.begin(), by_size.end(), 0);
      std::stable_sort(by_size.begin(), by_size.end(), [&](i64 a, i64 b) {
        return coff[cl_ids[a] + 1] - coff[cl_ids[a]] > coff[cl_ids[b] + 1] - coff[cl_ids[b]];
      });
      std::vector<i64> stack;
      for (i64 s0 : by_size) {
        if (placed[s0]) continue;
        stack.push_back(s0);
        while (!stack.empty()) {
          const i64 k = stack.back();
          stack.pop_back();
          if (placed[k]) continue;
          placed[k] = 1;
          corder.push_back(k);
          const auto& nb = cadj[k];          // strongest first -> pushed last
          for (size_t j = nb.size(); j-- > 0;)
            if (!placed[nb[j].second]) stack.push_back(nb[j].second);
        }
      }
    }
    std::vector<i64> cstart(ncl + 1, 0);
    for (i64 i = 0; i < ncl; ++i) {
      const i64 l = cl_ids[corder[i]];
      cstart[i + 1] = cstart[i] + (coff[l + 1] - coff[l]);
    }
    // Cuthill-McKee inside every cluster over its internal edges
    std::vector<char> seen(n, 0);
#pragma omp parallel for schedule(dynamic, 16)
    for (i64 i = 0; i < ncl; ++i) {
      const i64 l = cl_ids[corder[i]];
      const i64 b = coff[l], e = coff[l + 1];
      std::vector<i64> nodes(members.begin() + b, members.begin() + e);
      auto deg = [&](i64 v) { return rp[v + 1] - rp[v]; };
      std::stable_sort(nodes.begin(), nodes.end(), [&](i64 a, i64 c) { return deg(a) < deg(c); });
      std::vector<i64> q;
      q.reserve(nodes.size());
      std::vector<i64> nb;
      size_t next_root = 0, head = 0;
      while ((i64)q.size() < e - b) {
        while (seen[nodes[next_root]]) ++next_root;
        seen[nodes[next_root]] = 1;
        q.push_back(nodes[next_root]);
        while (head < q.size()) {
          const i64 v = q[head++];
          nb.clear();
          for (i64 x = rp[v]; x < rp[v + 1]; ++x) {
            const i64 u = col[x];
            if (lab[u] == l && !seen[u]) { seen[u] = 1; nb.push_back(u); }
          }
          std::stable_sort(nb.begin(), nb.end(), [&](i64 a, i64 c) { return deg(a) < deg(c); });
          q.insert(q.end(), nb.begin(), nb.end());
        }
      }
      for (size_t k = 0; k < q.size(); ++k) new_id[q[k]] = cstart[i] + (i64)k;
    }
  }
  return out;
}

// Refinement of an order by median smoothing (the 1-D barycenter heuristic with a
// robust centre): every node's key becomes the median position of itself and its
// neighbours, and the nodes are re-ranked by (key, previous position).  The median
// ignores the minority of long-range (inter-community) edges, so a locally banded
// structure -- which the cluster walk lays out only up to the cluster granularity --
// contracts to a narrow band around the diagonal; the re-ranking keeps positions a
// permutation, so nothing collapses.  O(iters * nnz) with a per-row nth_element.
py::array_t<i64> locality_refine(i64 n, I64Arr rowptr_a, I32Arr col_a, I64Arr new_id_a, int iters) {
  const i64* rp = rowptr_a.data();
  const i32* col = col_a.data();
  if (new_id_a.size() != n || rowptr_a.size() != n + 1) throw std::invalid_argument("locality_refine: sizes");
  py::array_t<i64> out(n);
  i64* pos = out.mutable_data();
  std::copy(new_id_a.data(), new_id_a.data() + n, pos);
  {
    py::gil_scoped_release nogil;
    const int nt = omp_get_max_threads();
    std::vector<std::vector<i64>> bufs(nt);
    std::vector<std::pair<i64, i64>> key(n);       // by previous position: (2 * median, position)
    std::vector<i64> order(n), node_at(n);
    for (int it = 0; it < iters; ++it) {
#pragma omp parallel for schedule(dynamic, 4096)
      for (i64 v = 0; v < n; ++v) {
        auto& b = bufs[omp_get_thread_num()];
        b.clear();
        b.push_back(pos[v]);
        for (i64 e = rp[v]; e < rp[v + 1]; ++e)
          if (col[e] != v) b.push_back(pos[col[e]]);
        const size_t h = b.size() / 2;
        std::nth_element(b.begin(), b.begin() + h, b.end());
        i64 med2 = 2 * b[h];
        if ((b.size() & 1) == 0) {              // even count: mean of the two middle values
          const i64 lo = *std::max_element(b.begin(), b.begin() + h);
          med2 = lo + b[h];
        }
        key[pos[v]] = {med2, pos[v]};
      }
      // previous positions sorted by key: order[p] = previous position of the node placed at p
      std::iota(order.begin(), order.end(), 0);
      for (i64 v = 0; v < n; ++v) node_at[pos[v]] = v;
      std::sort(order.begin(), order.end(), [&](i64 a, i64 b) { return key[a] < key[b]; });
      for (i64 p = 0; p < n; ++p) pos[node_at[order[p]]] = p;
    }
  }
  return out;
}

// Fraction of (non-loop) CSR entries whose endpoints are within w positions, for
// each window w in `windows`, under the order new_id (identity if empty).
std::vector<double> locality_stats(i64 n, I64Arr rowptr_a, I32Arr col_a, I64Arr new_id_a,
                                   std::vector<i64> windows) {
  const i64* rp = rowptr_a.data();
  const i32* col = col_a.data();
  const bool ident = new_id_a.size() == 0;
  const i64* nid = new_id_a.data();
  std::vector<double> out(windows.size(), 0.0);
  i64 total = 0;
  std::vector<i64> hits(windows.size(), 0);
  {
    py::gil_scoped_release nogil;
    const int nw = (int)windows.size();
#pragma omp parallel
    {
      std::vector<i64> h(nw, 0);
      i64 t = 0;
#pragma omp for schedule(static)
      for (i64 v = 0; v < n; ++v) {
        const i64 pv = ident ? v : nid[v];
        for (i64 e = rp[v]; e < rp[v + 1]; ++e) {
          const i64 u = col[e];
          if (u == v) continue;
          const i64 d = std::llabs((ident ? u : nid[u]) - pv);
          ++t;
          for (int k = 0; k < nw; ++k) h[k] += d <= windows[k];
        }
      }
#pragma omp critical
      {
        total += t;
        for (int k = 0; k < nw; ++k) hits[k] += h[k];
      }
    }
  }
  for (size_t k = 0; k < windows.size(); ++k) out[k] = total ? (double)hits[k] / (double)total : 0.0;
  return out;
}

// Apply a node permutation to a CSR: row new_id[v] of the result is row v of the
// input with its column ids mapped and sorted.  Returns (rowptr int64, col int32).
py::tuple permute_csr(i64 n, I64Arr rowptr_a, I32Arr col_a, I64Arr new_id_a) {
  const i64* rp = rowptr_a.data();
  const i32* col = col_a.data();
  const i64* nid = new_id_a.data();
  if (new_id_a.size() != n) throw std::invalid_argument("permute_csr: new_id size");
  py::array_t<i64> rp_out(n + 1);
  py::array_t<i32> col_out(rp[n]);
  i64* nrp = rp_out.mutable_data();
  i32* ncol = col_out.mutable_data();
  {
    py::gil_scoped_release nogil;
    std::vector<i64> old_of(n);
    for (i64 v = 0; v < n; ++v) old_of[nid[v]] = v;
    nrp[0] = 0;
    for (i64 r = 0; r < n; ++r) nrp[r + 1] = nrp[r] + (rp[old_of[r] + 1] - rp[old_of[r]]);
#pragma omp parallel for schedule(dynamic, 4096)
    for (i64 r = 0; r < n; ++r) {
      const i64 v = old_of[r];
      i32* dst = ncol + nrp[r];
      const i64 d = rp[v + 1] - rp[v];
      for (i64 k = 0; k < d; ++k) dst[k] = (i32)nid[col[rp[v] + k]];
      std::sort(dst, dst + d);
    }
  }
  return py::make_tuple(rp_out, col_out);
}

void register_reorder(py::module& m) {
  m.def("locality_order", &locality_order, py::arg("n"), py::arg("rowptr"), py::arg("col"),
        py::arg("lp_rounds") = 8, py::arg("max_cluster") = 4096, py::arg("seed") = 0);
  m.def("locality_refine", &locality_refine, py::arg("n"), py::arg("rowptr"), py::arg("col"),
        py::arg("new_id"), py::arg("iters") = 4);
  m.def("locality_stats", &locality_stats, py::arg("n"), py::arg("rowptr"), py::arg("col"),
        py::arg("new_id"), py::arg("windows"));
  m.def("permute_csr", &permute_csr, py::arg("n"), py::arg("rowptr"), py::arg("col"), py::arg("new_id"));
}
