// pt_bvh_build.cpp — host-side binned-SAH BVH builder, bit-exact with the
// reference's NumPy builder (src/render_server/taichi_renderer/
// sah_bvh_builder.py) under NumPy >= 2 scalar promotion (NEP 50): every
// quantity the reference keeps as np.float32 is a float here, Python float /
// int operands are rounded to float before the operation, and the evaluation
// order of each expression is the reference's. The reference builds a Python
// object per node in ~1.7 s for vol2_final_scene; this is a
// flat index-array build.
//
// Compiled with -ffp-contract=off (no FMA contraction) and without fast-math.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>

#include "../../include/ptmi.h"

namespace {

struct Box {
  float mn[3], mx[3];
};

struct Prim {
  int32_t type, idx;
  Box box;
  float c[3];
};

inline Box empty_box() {  // AABB.empty(), sah_bvh_builder.py:48-54
  Box b;
  for (int k = 0; k < 3; ++k) {
    b.mn[k] = std::numeric_limits<float>::infinity();
    b.mx[k] = -std::numeric_limits<float>::infinity();
  }
  return b;
}

// np.minimum / np.maximum: (a < b || isnan(a)) ? a : b, NaN propagating.
inline float npmin(float a, float b) { return (a < b || std::isnan(a)) ? a : b; }
inline float npmax(float a, float b) { return (a > b || std::isnan(a)) ? a : b; }

inline Box unite(const Box& a, const Box& b) {  // AABB.union, :41-46
  Box r;
  for (int k = 0; k < 3; ++k) {
    r.mn[k] = npmin(a.mn[k], b.mn[k]);
    r.mx[k] = npmax(a.mx[k], b.mx[k]);
  }
  return r;
}

inline float surface_area(const Box& b) {  // :26-29
  float e0 = b.mx[0] - b.mn[0], e1 = b.mx[1] - b.mn[1], e2 = b.mx[2] - b.mn[2];
  float s = e0 * e1 + e1 * e2;
  s = s + e2 * e0;
  return 2.0f * s;
}

inline void pad_to_minimums(Box& b) {  // :31-39
  const float delta = 0.0001f;
  const float half = 5e-05f;  // delta / 2.0 as a Python float, cast to f32
  for (int k = 0; k < 3; ++k) {
    if (b.mx[k] - b.mn[k] < delta) {
      float mid = (b.mn[k] + b.mx[k]) / 2.0f;
      b.mn[k] = mid - half;
      b.mx[k] = mid + half;
    }
  }
}

struct Node {
  Box box;
  int32_t left = -1, right = -1;  // builder node ids
  int32_t type = -1, idx = -1;
};

struct Builder {
  std::vector<Prim> prims;
  std::vector<Node> nodes;

  // _find_best_split, :243-336
  void best_split(const std::vector<int32_t>& ids, const Box& parent, int& best_axis, float& best_pos,
                  float& best_cost) {
    const int NB = 16;
    best_axis = 0;
    int best_bucket = 0;
    best_cost = std::numeric_limits<float>::infinity();
    for (int axis = 0; axis < 3; ++axis) {
      float minc = prims[ids[0]].c[axis], maxc = minc;
      for (size_t q = 1; q < ids.size(); ++q) {
        float v = prims[ids[q]].c[axis];
        if (v < minc) minc = v;
        if (v > maxc) maxc = v;
      }
      if (maxc - minc < 1e-10f) continue;
      int cnt[NB];
      Box bb[NB];
      for (int k = 0; k < NB; ++k) { cnt[k] = 0; bb[k] = empty_box(); }
      float extent = maxc - minc;
      for (int32_t id : ids) {
        float off = (prims[id].c[axis] - minc) / extent;
        int b = (int)(off * 16.0f);
        if (b > NB - 1) b = NB - 1;
        cnt[b] += 1;
        bb[b] = unite(bb[b], prims[id].box);
      }
      int lc[NB - 1], rc[NB - 1];
      Box lb[NB - 1], rb[NB - 1];
      Box run = empty_box();
      int rcount = 0;
      for (int i = 0; i < NB - 1; ++i) {
        rcount += cnt[i];
        run = unite(run, bb[i]);
        lc[i] = rcount;
        lb[i] = run;
      }
      run = empty_box();
      rcount = 0;
      for (int i = NB - 2; i >= 0; --i) {
        rcount += cnt[i + 1];
        run = unite(run, bb[i + 1]);
        rc[i] = rcount;
        rb[i] = run;
      }
      float psa = surface_area(parent);
      for (int i = 0; i < NB - 1; ++i) {
        if (lc[i] == 0 || rc[i] == 0) continue;
        float lsa = surface_area(lb[i]);
        float rsa = surface_area(rb[i]);
        // traverse_cost + (lsa/psa)*intersect_cost*nl + (rsa/psa)*intersect_cost*nr  (:314-316)
        float cost = 1.0f + (lsa / psa) * 1.5f * (float)lc[i];
        cost = cost + (rsa / psa) * 1.5f * (float)rc[i];
        if (cost < best_cost) {
          best_cost = cost;
          best_axis = axis;
          best_bucket = i;
        }
      }
    }
    if (best_cost < std::numeric_limits<float>::infinity()) {
      float minc = prims[ids[0]].c[best_axis], maxc = minc;
      for (size_t q = 1; q < ids.size(); ++q) {
        float v = prims[ids[q]].c[best_axis];
        if (v < minc) minc = v;
        if (v > maxc) maxc = v;
      }
      float extent = maxc - minc;
      float step = ((float)(best_bucket + 1) * extent) / 16.0f;
      best_pos = minc + step;
    } else {  // median on axis 0 (:330-334)
      std::vector<int32_t> s(ids);
      std::stable_sort(s.begin(), s.end(), [&](int32_t a, int32_t b) { return prims[a].c[0] < prims[b].c[0]; });
      best_pos = prims[s[s.size() / 2]].c[0];
      best_axis = 0;
    }
  }

  // _build_recursive, :179-241. Returns builder node id.
  int32_t build(std::vector<int32_t>& ids) {
    int32_t me = (int32_t)nodes.size();
    nodes.emplace_back();
    Box bb = empty_box();
    for (int32_t id : ids) bb = unite(bb, prims[id].box);
    nodes[me].box = bb;
    if (ids.size() == 1) {
      nodes[me].type = prims[ids[0]].type;
      nodes[me].idx = prims[ids[0]].idx;
      return me;
    }
    int axis;
    float pos, cost;
    best_split(ids, bb, axis, pos, cost);
    std::vector<int32_t> L, R;
    L.reserve(ids.size());
    R.reserve(ids.size());
    for (int32_t id : ids) (prims[id].c[axis] < pos ? L : R).push_back(id);
    if (L.empty() || R.empty()) {  // :226-231 median fallback
      std::vector<int32_t> s(ids);
      std::stable_sort(s.begin(), s.end(),
                       [&](int32_t a, int32_t b) { return prims[a].c[axis] < prims[b].c[axis]; });
      size_t mid = s.size() / 2;
      L.assign(s.begin(), s.begin() + (long)mid);
      R.assign(s.begin() + (long)mid, s.end());
    }
    std::vector<int32_t>().swap(ids);
    int32_t l = build(L);
    int32_t r = build(R);
    nodes[me].left = l;
    nodes[me].right = r;
    return me;
  }
};

}  // namespace

extern "C" int ptmi_bvh_build_sah(const float* spheres, int32_t ns, const float* quads, int32_t nq, const float* tris,
                                  int32_t nt, float* bbox_min, float* bbox_max, int32_t* left, int32_t* right,
                                  int32_t* parent, int32_t* prim_type, int32_t* prim_idx, int32_t* n_nodes) {
  if (ns < 0 || nq < 0 || nt < 0 || !n_nodes) return PTMI_EINVAL;
  if ((ns && !spheres) || (nq && !quads) || (nt && !tris)) return PTMI_EINVAL;
  int64_t np = (int64_t)ns + nq + nt;
  *n_nodes = 0;
  if (np == 0) return PTMI_OK;
  if (np > (1 << 27)) return PTMI_ECAPACITY;
  if (!bbox_min || !bbox_max || !left || !right || !parent || !prim_type || !prim_idx) return PTMI_EINVAL;
  Builder B;
  B.prims.reserve((size_t)np);
  for (int32_t i = 0; i < ns; ++i) {  // add_sphere, :104-116
    const float* s = spheres + 4 * i;
    Prim p;
    p.type = 0;
    p.idx = i;
    for (int k = 0; k < 3; ++k) {
      p.box.mn[k] = s[k] - s[3];
      p.box.mx[k] = s[k] + s[3];
      p.c[k] = s[k];
    }
    B.prims.push_back(p);
  }
  for (int32_t i = 0; i < nq; ++i) {  // add_quad, :118-143
    const float* q = quads + 9 * i;
    Prim p;
    p.type = 2;
    p.idx = i;
    for (int k = 0; k < 3; ++k) {
      float Q = q[k], u = q[3 + k], v = q[6 + k];
      float c1 = Q + u, c2 = Q + v, c3 = (Q + u) + v;
      float mn = Q, mx = Q;
      for (float c : {c1, c2, c3}) {
        mn = npmin(mn, c);
        mx = npmax(mx, c);
      }
      p.box.mn[k] = mn;
      p.box.mx[k] = mx;
      p.c[k] = (Q + 0.5f * u) + 0.5f * v;
    }
    pad_to_minimums(p.box);
    B.prims.push_back(p);
  }
  for (int32_t i = 0; i < nt; ++i) {  // add_triangle, :145-165
    const float* t = tris + 9 * i;
    Prim p;
    p.type = 1;
    p.idx = i;
    for (int k = 0; k < 3; ++k) {
      float a = t[k], b = t[3 + k], c = t[6 + k];
      p.box.mn[k] = npmin(npmin(a, b), c);
      p.box.mx[k] = npmax(npmax(a, b), c);
      p.c[k] = ((a + b) + c) / 3.0f;
    }
    pad_to_minimums(p.box);
    B.prims.push_back(p);
  }
  B.nodes.reserve((size_t)(2 * np));
  std::vector<int32_t> ids((size_t)np);
  for (int64_t i = 0; i < np; ++i) ids[(size_t)i] = (int32_t)i;
  int32_t root = B.build(ids);
  // flatten, :338-418: preorder, left before right.
  std::vector<int32_t> flat_of(B.nodes.size(), -1);
  struct Item { int32_t node, parent; };
  std::vector<Item> st;
  st.push_back({root, -1});
  int32_t n = 0;
  while (!st.empty()) {
    Item it = st.back();
    st.pop_back();
    int32_t me = n++;
    flat_of[(size_t)it.node] = me;
    const Node& nd = B.nodes[(size_t)it.node];
    for (int k = 0; k < 3; ++k) {
      bbox_min[3 * me + k] = nd.box.mn[k];
      bbox_max[3 * me + k] = nd.box.mx[k];
    }
    parent[me] = it.parent;
    prim_type[me] = nd.type;
    prim_idx[me] = nd.idx;
    left[me] = -1;
    right[me] = -1;
    if (nd.left >= 0) {
      st.push_back({nd.right, me});
      st.push_back({nd.left, me});
    }
  }
  for (size_t k = 0; k < B.nodes.size(); ++k) {
    const Node& nd = B.nodes[k];
    if (nd.left >= 0) {
      int32_t me = flat_of[k];
      left[me] = flat_of[(size_t)nd.left];
      right[me] = flat_of[(size_t)nd.right];
    }
  }
  *n_nodes = n;
  return PTMI_OK;
}
