// selector_dev.hpp — QuerySelector on the device (QuerySelector.java:76-374), shared by the general window
// path (window_gen.hip) and the NFA's pattern selector stage (nfa.hip).
//
// Input: M items in processing order -- (type, timestamp, value row, partition instance, chunk ordinal) --
// and the pre-selector values of their rows (GwdVals).  DevSelector::run
//   * hashes each item's aggregator key (group-by values, plus the instance when partitioned), radix-sorts
//     the items by it (stable) into group segments and checks that equal hashes carry equal keys;
//   * looks up each group's carried aggregator state in the SelectorStage's state store (host, O(groups));
//   * sum / count / avg: segmented inclusive scans in exact integer arithmetic (a RESET item opens a new
//     segment); min / max: one lane per group replaying the deque (window_dev.hpp kernels);
//   * output attributes and having per item (k_gwd_out), a flagged select of the rows that pass;
//   * writes the groups' final states back to the state store.
// It returns false -- having changed nothing -- when a group-key hash collides or a double sum could round;
// the caller then runs the host SelectorStage on the same items.  DevSelector::batch applies the per-chunk
// batching to the selected rows: last row per group in first-appearance order, the last row of an
// aggregating chunk, or every row; order by / offset / limit on the host over the (few) rows of a chunk.
#pragma once
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cmath>
#include <cstring>
#include <functional>
#include <unordered_map>
#include <vector>

#include "runtime.hpp"
#include "selector.hpp"
#include "window_dev.hpp"

namespace sg {

struct DevSelRows {
  int64_t P = 0;                  // selected rows, in item order
  int nout = 0;
  std::vector<int64_t> ts;
  std::vector<int32_t> meta;      // [P][3]: item type, chunk ordinal, group
  std::vector<int64_t> raw;       // [P][nout]
  std::vector<uint8_t> nul;
  int32_t ord(int64_t r) const { return meta[(size_t)(3 * r + 1)]; }
  SelOut row(int64_t r) const {
    SelOut so;
    so.ts = ts[(size_t)r];
    so.expired = meta[(size_t)(3 * r)] == GI_EXP;
    so.raw.assign(raw.begin() + r * nout, raw.begin() + (r + 1) * nout);
    so.nul.assign(nul.begin() + r * nout, nul.begin() + (r + 1) * nout);
    return so;
  }
};

struct DevSelector {
  DBuf<uint8_t> tmp, pass, onul, an, mvn0, fin_mvn, o_nul;
  DBuf<uint64_t> hkey, shkey;
  DBuf<int64_t> out, av, xc, nc, X, N, init_x, init_n, fin_x, fin_n, keys, o_ts, o_raw, dq_in, mv0, wo, ws, fin_mv;
  DBuf<int32_t> iota, sidx, head, head2, gnum, seg2, rflag, rcnt, rep, gid, bad, pidx, nP, o_meta, gstart, dq_off,
      fin_h, fin_t, need;
  DBuf<unsigned long long> mx;
  DBuf<Prog> progs, having;
  bool progs_up = false;

  static unsigned gdim(int64_t n) { return (unsigned)std::max<int64_t>(1, (n + GWD_B - 1) / GWD_B); }
  void cub_tmp(size_t b) { tmp.reserve(std::max<size_t>(b, 1), false); }
  template <class T>
  void incl_sum(const T* in, T* o, int64_t n, hipStream_t s) {
    size_t tb = 0;
    SG_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, tb, in, o, (int)n, s));
    cub_tmp(tb);
    SG_HIP(hipcub::DeviceScan::InclusiveSum(tmp.p, tb, in, o, (int)n, s));
  }
  template <class K, class T>
  void incl_sum_by_key(const K* keys_, const T* in, T* o, int64_t n, hipStream_t s) {
    size_t tb = 0;
    SG_HIP(hipcub::DeviceScan::InclusiveSumByKey(nullptr, tb, keys_, in, o, (int)n, hipcub::Equality(), s));
    cub_tmp(tb);
    SG_HIP(hipcub::DeviceScan::InclusiveSumByKey(tmp.p, tb, keys_, in, o, (int)n, hipcub::Equality(), s));
  }
  template <class T>
  static void h2d(DBuf<T>& d, const T* h, size_t n, hipStream_t s) {
    d.reserve(std::max<size_t>(n, 1), false);
    if (n) SG_HIP(hipMemcpyAsync(d.p, h, n * sizeof(T), hipMemcpyHostToDevice, s));
  }
  template <class T>
  static void d2h(T* h, const T* d, size_t n, hipStream_t s) {
    if (n) SG_HIP(hipMemcpyAsync(h, d, n * sizeof(T), hipMemcpyDeviceToHost, s));
  }

  // `partitioned`: the instance is part of the aggregator key, part_of(instance) its SelIn.part value;
  // `R`: value rows (exactness statistics run over all of them)
  bool run(const SelSpec& sp, SelectorStage& sel, bool partitioned, int64_t M, const GwdItems& it, const GwdVals& vals,
           int64_t R, const std::function<int64_t(int32_t)>& part_of, hipStream_t s, DevSelRows& res) {
    const int naggs = (int)sp.aggs.size();
    const bool gb = !sp.group.empty();
    const bool grouping = gb || (naggs > 0 && partitioned);
    const int nout = (int)sp.akind.size();
    res = DevSelRows();
    res.nout = nout;
    if (M <= 0) return true;
    int64_t G = 0;
    std::vector<int32_t> shift((size_t)std::max(naggs, 1), 0);
    std::vector<std::vector<AggSt>> gst;        // per group: the carried states (lookup) -> final states
    std::vector<AggSt> mm_fin;                  // [group][aggregator] final min / max states
    std::vector<SelectorStage::GKey> gkeys;
    GwdSelArgs sa;
    std::memset(&sa, 0, sizeof(sa));
    const size_t m = (size_t)M;
    hkey.reserve(m, false); shkey.reserve(m, false); sidx.reserve(m, false); head.reserve(m, false);
    head2.reserve(m, false); gnum.reserve(m, false); seg2.reserve(m, false); rflag.reserve(m, false);
    rcnt.reserve(m, false); gid.reserve(m, false); rep.reserve(m, false); bad.reserve(1, false);
    iota.reserve(m, false); gstart.reserve(m + 1, false);
    sa.M = M; sa.it = it; sa.vals = vals; sa.ng = gb ? (int32_t)sp.group.size() : 0;
    for (int g = 0; g < sa.ng; g++) sa.gcol[g] = sp.group[(size_t)g];
    sa.keyed_lid = partitioned && grouping;
    sa.hkey = hkey.p; sa.iota = iota.p; sa.head = head.p; sa.head2 = head2.p; sa.gnum = gnum.p;
    sa.rep = rep.p; sa.bad = bad.p; sa.gid = gid.p; sa.gstart = gstart.p;
    hipLaunchKernelGGL(k_gwd_hash, dim3(gdim(M)), dim3(GWD_B), 0, s, sa);
    if (grouping) {
      size_t tb = 0;
      SG_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, hkey.p, shkey.p, iota.p, sidx.p, (int)M, 0, 64, s));
      cub_tmp(tb);
      SG_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb, hkey.p, shkey.p, iota.p, sidx.p, (int)M, 0, 64, s));
    } else {
      SG_HIP(hipMemcpyAsync(shkey.p, hkey.p, m * 8, hipMemcpyDeviceToDevice, s));
      SG_HIP(hipMemcpyAsync(sidx.p, iota.p, m * 4, hipMemcpyDeviceToDevice, s));
    }
    sa.shkey = shkey.p; sa.sidx = sidx.p;
    hipLaunchKernelGGL(k_gwd_heads, dim3(gdim(M)), dim3(GWD_B), 0, s, sa, rflag.p);
    incl_sum(head.p, gnum.p, M, s);
    incl_sum(head2.p, seg2.p, M, s);
    SG_HIP(hipMemsetAsync(bad.p, 0, 4, s));
    hipLaunchKernelGGL(k_gwd_groups, dim3(gdim(M)), dim3(GWD_B), 0, s, sa);
    hipLaunchKernelGGL(k_gwd_verify, dim3(gdim(M)), dim3(GWD_B), 0, s, sa);
    int32_t hb[2] = {0, 0};
    d2h(&hb[0], gnum.p + M - 1, 1, s);
    d2h(&hb[1], bad.p, 1, s);
    SG_HIP(hipStreamSynchronize(s));
    G = hb[0];
    if (hb[1]) return false;                                  // hash collision of two group keys
    SG_HIP(hipGetLastError());
    if (naggs > 0) {
      // the carried states of the groups
      const int w = 2 * sa.ng + 1;
      std::vector<int64_t> hk((size_t)G * w);
      keys.reserve((size_t)G * w, false);
      hipLaunchKernelGGL(k_gwd_repkeys, dim3(gdim(G)), dim3(GWD_B), 0, s, sa, G, keys.p);
      d2h(hk.data(), keys.p, hk.size(), s);
      SG_HIP(hipStreamSynchronize(s));
      gkeys.resize((size_t)G);
      gst.resize((size_t)G);
      for (int64_t g = 0; g < G; g++) {
        SelectorStage::GKey k(hk.begin() + g * w, hk.begin() + g * w + 2 * sa.ng);
        if (sp.partitioned) k.push_back(part_of((int32_t)hk[(size_t)(g * w + 2 * sa.ng)]));
        const std::vector<AggSt>* st0 = sel.state_find(k);
        gst[(size_t)g] = st0 ? *st0 : std::vector<AggSt>((size_t)naggs);
        gkeys[(size_t)g] = std::move(k);
      }
      // exactness: every sum the reference forms stays an exact double
      need.reserve(1, false); mx.reserve(1, false);
      for (int a = 0; a < naggs; a++) {
        const SelAgg& A = sp.aggs[(size_t)a];
        if (A.k == SA_COUNT || A.k == SA_MIN || A.k == SA_MAX) continue;
        int32_t nd = 0;
        unsigned long long mxb = 0;
        SG_HIP(hipMemsetAsync(need.p, 0, 4, s));
        SG_HIP(hipMemsetAsync(mx.p, 0, 8, s));
        if (R > 0) hipLaunchKernelGGL(k_gwd_xstat, dim3(gdim(R)), dim3(GWD_B), 0, s, R, vals, (int32_t)A.arg,
                                      (int32_t)A.in_t, need.p, mx.p);
        d2h(&nd, need.p, 1, s);
        d2h(&mxb, mx.p, 1, s);
        SG_HIP(hipStreamSynchronize(s));
        double mxv;
        std::memcpy(&mxv, &mxb, 8);
        const bool long_sum = A.k == SA_SUM && (A.in_t == T_INT || A.in_t == T_LONG);
        double init_max = 0;
        for (auto& v : gst) {
          const double x = long_sum ? std::fabs((double)v[(size_t)a].lsum) : std::fabs(v[(size_t)a].dsum);
          init_max = std::max(init_max, x);
          if (!long_sum && v[(size_t)a].dsum != 0.0) {
            int e2;
            const double fm = std::frexp(v[(size_t)a].dsum, &e2);
            const uint64_t bits = (uint64_t)std::ldexp(std::fabs(fm), 53);
            const int lsb = e2 - 53 + __builtin_ctzll(bits);
            nd = std::max(nd, lsb < 0 ? -lsb : 0);
          }
        }
        if (nd > 60 || (long_sum && nd > 0)) return false;
        const int S = long_sum ? 0 : nd;
        if ((init_max + (double)M * mxv) * std::ldexp(1.0, S) >= 9007199254740992.0) return false;
        shift[(size_t)a] = S;
      }
      SG_HIP(hipGetLastError());
    }
    // nothing has changed yet: from here on the selector completes on the device
    if (naggs > 0) {
      incl_sum_by_key(gnum.p, rflag.p, rcnt.p, M, s);
      xc.reserve(m, false); nc.reserve(m, false); X.reserve(m, false); N.reserve(m, false);
      av.reserve(m * naggs, false); an.reserve(m * naggs, false);
      init_x.reserve((size_t)G, false); init_n.reserve((size_t)G, false);
      fin_x.reserve((size_t)G * naggs, false); fin_n.reserve((size_t)G * naggs, false);
      mm_fin.assign((size_t)G * naggs, AggSt());
      std::vector<int64_t> ix((size_t)G), in_((size_t)G);
      std::vector<int32_t> hgs;                          // group starts (min / max lanes)
      for (int a = 0; a < naggs; a++) {
        const SelAgg& A = sp.aggs[(size_t)a];
        if (A.k == SA_MIN || A.k == SA_MAX) {
          if (hgs.empty()) {
            const int32_t mm = (int32_t)M;
            SG_HIP(hipMemcpyAsync(gstart.p + G, &mm, 4, hipMemcpyHostToDevice, s));
            hgs.resize((size_t)G + 1);
            d2h(hgs.data(), gstart.p, (size_t)G + 1, s);
            SG_HIP(hipStreamSynchronize(s));
          }
          std::vector<int32_t> dqo((size_t)G + 1, 0);
          std::vector<int64_t> dqv, hmv((size_t)G), hwo((size_t)G + 1, 0);
          std::vector<uint8_t> hmvn((size_t)G);
          for (int64_t g = 0; g < G; g++) {
            const AggSt& st = gst[(size_t)g][(size_t)a];
            dqo[(size_t)g] = (int32_t)dqv.size();
            dqv.insert(dqv.end(), st.dq.begin(), st.dq.end());
            hmv[(size_t)g] = st.mv; hmvn[(size_t)g] = st.mv_null;
            hwo[(size_t)g + 1] = hwo[(size_t)g] + (int64_t)st.dq.size() + (hgs[(size_t)g + 1] - hgs[(size_t)g]);
          }
          dqo[(size_t)G] = (int32_t)dqv.size();
          h2d(dq_off, dqo.data(), dqo.size(), s);
          h2d(dq_in, dqv.data(), dqv.size(), s);
          h2d(mv0, hmv.data(), hmv.size(), s);
          h2d(mvn0, hmvn.data(), hmvn.size(), s);
          h2d(wo, hwo.data(), hwo.size(), s);
          ws.reserve((size_t)std::max<int64_t>(hwo[(size_t)G], 1), false);
          fin_mv.reserve((size_t)G, false); fin_mvn.reserve((size_t)G, false);
          fin_h.reserve((size_t)G, false); fin_t.reserve((size_t)G, false);
          GwdMinMaxArgs ma;
          ma.G = G; ma.gstart = gstart.p; ma.sidx = sidx.p; ma.it = it; ma.vals = vals;
          ma.arg = A.arg; ma.in_t = (int32_t)A.in_t; ma.is_min = A.k == SA_MIN; ma.track = A.track;
          ma.dq_off = dq_off.p; ma.dq_in = dq_in.p; ma.mv0 = mv0.p; ma.mvn0 = mvn0.p; ma.wo = wo.p;
          ma.ws = ws.p; ma.av = av.p + m * a; ma.an = an.p + m * a; ma.fin_mv = fin_mv.p;
          ma.fin_mvn = fin_mvn.p; ma.fin_h = fin_h.p; ma.fin_t = fin_t.p;
          hipLaunchKernelGGL(k_gwd_minmax, dim3((unsigned)((G + 63) / 64)), dim3(64), 0, s, ma);
          SG_HIP(hipGetLastError());
          std::vector<int64_t> fmv((size_t)G), wsh((size_t)hwo[(size_t)G]);
          std::vector<uint8_t> fmvn((size_t)G);
          std::vector<int32_t> fh((size_t)G), ft((size_t)G);
          d2h(fmv.data(), fin_mv.p, (size_t)G, s);
          d2h(fmvn.data(), fin_mvn.p, (size_t)G, s);
          d2h(fh.data(), fin_h.p, (size_t)G, s);
          d2h(ft.data(), fin_t.p, (size_t)G, s);
          if (A.track) d2h(wsh.data(), ws.p, wsh.size(), s);
          SG_HIP(hipStreamSynchronize(s));
          for (int64_t g = 0; g < G; g++) {                 // the final states, stored with the others below
            AggSt& st = mm_fin[(size_t)g * naggs + a];
            st.mv = fmv[(size_t)g]; st.mv_null = fmvn[(size_t)g] != 0;
            st.dq.clear();
            if (A.track)
              for (int32_t k = fh[(size_t)g]; k < ft[(size_t)g]; k++) st.dq.push_back(wsh[(size_t)(hwo[(size_t)g] + k)]);
          }
          continue;
        }
        const bool long_sum = A.k == SA_SUM && (A.in_t == T_INT || A.in_t == T_LONG);
        for (int64_t g = 0; g < G; g++) {
          const AggSt& v = gst[(size_t)g][(size_t)a];
          in_[(size_t)g] = v.count;
          ix[(size_t)g] = A.k == SA_COUNT ? 0 : long_sum ? v.lsum : (int64_t)std::ldexp(v.dsum, shift[(size_t)a]);
        }
        h2d(init_x, ix.data(), (size_t)G, s);
        h2d(init_n, in_.data(), (size_t)G, s);
        GwdAgg ga{(int32_t)A.k, (int32_t)A.arg, (int32_t)A.in_t, shift[(size_t)a]};
        hipLaunchKernelGGL(k_gwd_contrib, dim3(gdim(M)), dim3(GWD_B), 0, s, sa, ga, xc.p, nc.p);
        incl_sum_by_key(seg2.p, xc.p, X.p, M, s);
        incl_sum_by_key(seg2.p, nc.p, N.p, M, s);
        GwdAggOutArgs oa;
        oa.M = M; oa.sidx = sidx.p; oa.head = gnum.p; oa.rcnt = rcnt.p; oa.X = X.p; oa.N = N.p;
        oa.init_x = init_x.p; oa.init_n = init_n.p; oa.A = ga; oa.av = av.p + m * a; oa.an = an.p + m * a;
        oa.fin_x = fin_x.p + (size_t)G * a; oa.fin_n = fin_n.p + (size_t)G * a;
        hipLaunchKernelGGL(k_gwd_aggout, dim3(gdim(M)), dim3(GWD_B), 0, s, oa);
        SG_HIP(hipStreamSynchronize(s));   // init_x / init_n are reused by the next aggregator
      }
    }
    if (!progs_up) {
      progs.reserve(sp.host.size() + 1, false);
      having.reserve(1, false);
      if (!sp.host.empty()) SG_HIP(hipMemcpyAsync(progs.p, sp.host.data(), sp.host.size() * sizeof(Prog), hipMemcpyHostToDevice, s));
      SG_HIP(hipMemcpyAsync(having.p, &sp.having, sizeof(Prog), hipMemcpyHostToDevice, s));
      progs_up = true;
    }
    out.reserve(m * std::max(nout, 1), false); onul.reserve(m * std::max(nout, 1), false); pass.reserve(m, false);
    GwdOutArgs ua;
    ua.M = M; ua.it = it; ua.vals = vals; ua.naggs = naggs;
    ua.av = naggs ? av.p : nullptr; ua.an = naggs ? an.p : nullptr; ua.nout = nout;
    for (int k = 0; k < nout; k++) { ua.akind[k] = sp.akind[(size_t)k]; ua.aidx[k] = sp.aidx[(size_t)k]; }
    ua.progs = progs.p; ua.has_having = sp.has_having; ua.having = having.p;
    ua.current_on = sp.current_on; ua.expired_on = sp.expired_on;
    ua.out = out.p; ua.onul = onul.p; ua.pass = pass.p;
    hipLaunchKernelGGL(k_gwd_out, dim3(gdim(M)), dim3(GWD_B), 0, s, ua);
    SG_HIP(hipGetLastError());
    pidx.reserve(m, false);
    {
      hipcub::CountingInputIterator<int32_t> idx(0);
      size_t tb = 0;
      nP.reserve(1, false);
      SG_HIP(hipcub::DeviceSelect::Flagged(nullptr, tb, idx, pass.p, pidx.p, nP.p, (int)M, s));
      cub_tmp(tb);
      SG_HIP(hipcub::DeviceSelect::Flagged(tmp.p, tb, idx, pass.p, pidx.p, nP.p, (int)M, s));
      int32_t np = 0;
      d2h(&np, nP.p, 1, s);
      SG_HIP(hipStreamSynchronize(s));
      res.P = np;
    }
    const int64_t P = res.P;
    if (P > 0) {
      const size_t p = (size_t)P;
      o_ts.reserve(p, false); o_meta.reserve(3 * p, false);
      o_raw.reserve(p * std::max(nout, 1), false); o_nul.reserve(p * std::max(nout, 1), false);
      hipLaunchKernelGGL(k_gwd_pack_out, dim3(gdim(P)), dim3(GWD_B), 0, s, P, pidx.p, it, grouping ? gid.p : nullptr,
                         nout, out.p, onul.p, o_ts.p, o_meta.p, o_raw.p, o_nul.p);
      res.ts.resize(p); res.meta.resize(3 * p); res.raw.resize(p * nout); res.nul.resize(p * nout);
      d2h(res.ts.data(), o_ts.p, p, s);
      d2h(res.meta.data(), o_meta.p, 3 * p, s);
      d2h(res.raw.data(), o_raw.p, p * nout, s);
      d2h(res.nul.data(), o_nul.p, p * nout, s);
    }
    if (naggs > 0) {
      std::vector<int64_t> fx((size_t)G * naggs), fn((size_t)G * naggs);
      d2h(fx.data(), fin_x.p, fx.size(), s);
      d2h(fn.data(), fin_n.p, fn.size(), s);
      SG_HIP(hipStreamSynchronize(s));
      for (int64_t g = 0; g < G; g++) {
        std::vector<AggSt>& v = gst[(size_t)g];
        for (int a = 0; a < naggs; a++) {
          const SelAgg& A = sp.aggs[(size_t)a];
          if (A.k == SA_MIN || A.k == SA_MAX) { v[(size_t)a] = std::move(mm_fin[(size_t)g * naggs + a]); continue; }
          const int64_t x = fx[(size_t)a * G + g], c = fn[(size_t)a * G + g];
          AggSt st;
          st.count = c;
          if (A.k == SA_SUM && (A.in_t == T_INT || A.in_t == T_LONG)) st.lsum = x;
          else if (A.k != SA_COUNT) st.dsum = std::ldexp((double)x, -shift[(size_t)a]);
          v[(size_t)a] = st;
        }
        if ((gb || sp.partitioned) && sel.destroyable(v)) sel.state_erase(gkeys[(size_t)g]);
        else sel.state_put(gkeys[(size_t)g], std::move(v));
      }
    }
    SG_HIP(hipStreamSynchronize(s));
    return true;
  }

  // QuerySelector's batching of one output chunk: selected rows [q, qe) (one chunk ordinal)
  static void batch(const SelSpec& sp, const SelectorStage& sel, const DevSelRows& r, int64_t q, int64_t qe,
                    std::vector<SelOut>& so) {
    so.clear();
    if (!sp.group.empty()) {   // last row of each group, in the order of the groups' first rows
      std::vector<std::pair<int32_t, int64_t>> firsts;   // (group, last row)
      std::unordered_map<int32_t, size_t> at;
      for (int64_t x = q; x < qe; x++) {
        const int32_t g = r.meta[(size_t)(3 * x + 2)];
        auto f = at.find(g);
        if (f == at.end()) { at.emplace(g, firsts.size()); firsts.push_back({g, x}); }
        else firsts[f->second].second = x;
      }
      for (auto& fr : firsts) so.push_back(r.row(fr.second));
      sel.finish_chunk(so);
    } else if (!sp.aggs.empty()) {
      if (sp.offset <= 0 && sp.limit != 0) so.push_back(r.row(qe - 1));
    } else {
      for (int64_t x = q; x < qe; x++) so.push_back(r.row(x));
      sel.finish_chunk(so);
    }
  }
};

}  // namespace sg
