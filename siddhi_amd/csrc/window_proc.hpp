// window_proc.hpp — the reference's window processors on one instance, restated once and shared by the
// general single-stream path (window_gen.hip) and the window extension ABI (ext.hip, sg_window_*):
//   LengthWindowProcessor.process      CORE/query/processor/stream/window/LengthWindowProcessor.java:106-141
//   TimeWindowProcessor.process        TimeWindowProcessor.java:133-169 (notifyAt(ts + T) per new timestamp)
//   LengthBatchWindowProcessor.process LengthBatchWindowProcessor.java:154-351 (both modes)
// Items carry an opaque payload P (pre-selector values in window_gen, event ids in the extension ABI);
// every output chunk goes to emit(std::vector<WinItem<P>>&), in the reference's order.
#pragma once
#include <cstdint>
#include <deque>
#include <vector>

namespace sg {

enum WinKind { WK_NONE = 0, WK_LENGTH, WK_TIME, WK_BATCH };
enum WinEvType { WE_CURRENT = 0, WE_EXPIRED = 1, WE_RESET = 3 };   // ComplexEvent.Type (as SelEvType)

template <class P>
struct WinItem {
  int type;
  int64_t ts;
  P val;
};

struct WinSpec {
  int kind = WK_NONE;
  int64_t L = 0;               // length / batch count, or time span (ms)
  bool stream_current = false; // lengthBatch(L, true)
  bool expired_on = false;     // the query outputs expired events (outputExpectsExpiredEvents)
};

template <class P>
struct WinState {
  std::deque<WinItem<P>> q;           // length / time: the expired-event queue
  int64_t count = 0;
  int64_t last_ts = INT64_MIN;        // time: TimeWindowProcessor.lastTimestamp
  std::deque<int64_t> timers;         // time: Scheduler FIFO of notifyAt deadlines
  std::vector<WinItem<P>> cur, exq;   // lengthBatch
  bool has_reset = false;
  WinItem<P> reset{};
};

template <class P>
inline WinItem<P> win_expired(WinItem<P> x, int64_t ts) {
  x.type = WE_EXPIRED;
  x.ts = ts;
  return x;
}

// TimeWindowProcessor: expire every held event with ts - now + T <= 0 (re-stamped with now)
template <class P>
inline void win_expire_time(const WinSpec& sp, WinState<P>& I, int64_t now, std::vector<WinItem<P>>& o) {
  while (!I.q.empty() && I.q.front().ts - now + sp.L <= 0) {
    WinItem<P> x = I.q.front();
    I.q.pop_front();
    x.ts = now;
    o.push_back(x);
  }
}

// lengthBatch at a batch boundary: the previous batch as EXPIRED events, then the RESET event
template <class P>
inline void win_flush_batch_expired(const WinSpec& sp, WinState<P>& I, int64_t now, std::vector<WinItem<P>>& o) {
  if (sp.expired_on && !I.exq.empty()) {
    for (WinItem<P>& x : I.exq) { x.ts = now; o.push_back(x); }
    I.exq.clear();
  }
  if (I.has_reset) {
    I.reset.ts = now;
    o.push_back(I.reset);
    I.has_reset = false;
  }
}

// the window processor on the CURRENT events of one chunk (app clock `now`); notify() after a time
// window's notifyAt (the instance's Scheduler state becomes live)
template <class P, class Emit, class Notify>
void win_process(const WinSpec& sp, WinState<P>& I, const std::vector<WinItem<P>>& evs, int64_t now, Emit&& emit,
                 Notify&& notify) {
  std::vector<WinItem<P>> o;
  switch (sp.kind) {
    case WK_NONE: {
      std::vector<WinItem<P>> c = evs;
      emit(c);
      return;
    }
    case WK_LENGTH:
      for (const WinItem<P>& e : evs) {
        if (I.count < sp.L) {
          I.count++;
          I.q.push_back(win_expired(e, e.ts));
          o.push_back(e);
        } else if (!I.q.empty()) {
          o.push_back(win_expired(I.q.front(), now));
          I.q.pop_front();
          o.push_back(e);
          I.q.push_back(win_expired(e, e.ts));
        } else {   // length(0): the event passes through, expires and resets at once
          o.push_back(e);
          o.push_back(win_expired(e, e.ts));
          WinItem<P> r = e;
          r.type = WE_RESET;
          o.push_back(r);
        }
      }
      emit(o);
      return;
    case WK_TIME:
      for (const WinItem<P>& e : evs) {
        win_expire_time(sp, I, now, o);
        I.q.push_back(win_expired(e, e.ts));
        if (I.last_ts < e.ts) {        // Scheduler.notifyAt
          I.timers.push_back(e.ts + sp.L);
          I.last_ts = e.ts;
          notify();
        }
        o.push_back(e);
      }
      emit(o);
      return;
    default:
      break;
  }
  // lengthBatch: every event is its own processor call, hence its own (possibly empty) output chunk
  for (const WinItem<P>& e : evs) {
    o.clear();
    if (sp.L == 0) {
      o.push_back(e);
      if (sp.expired_on) o.push_back(win_expired(e, now));
      WinItem<P> r = e;
      r.type = WE_RESET;
      r.ts = now;
      o.push_back(r);
    } else {
      if (!I.has_reset) { I.reset = e; I.reset.type = WE_RESET; I.has_reset = true; }
      if (sp.stream_current) {
        I.count++;
        if (I.count == sp.L + 1) {
          win_flush_batch_expired(sp, I, now, o);
          I.count = 1;
        }
        o.push_back(e);
        if (sp.expired_on) I.exq.push_back(win_expired(e, e.ts));
      } else {
        I.cur.push_back(e);
        I.count++;
        if (I.count == sp.L) {
          win_flush_batch_expired(sp, I, now, o);
          if (!I.cur.empty()) {
            if (sp.expired_on)
              for (const WinItem<P>& x : I.cur) I.exq.push_back(win_expired(x, x.ts));
            for (const WinItem<P>& x : I.cur) o.push_back(x);
            I.cur.clear();
          }
          I.count = 0;
        }
      }
    }
    emit(o);
  }
}

// Scheduler.onTimeChange for a firing time-window state: each due deadline is one TIMER chunk
template <class P, class Emit>
void win_drain(const WinSpec& sp, WinState<P>& I, int64_t now, Emit&& emit) {
  while (!I.timers.empty() && I.timers.front() - now <= 0) {
    I.timers.pop_front();
    std::vector<WinItem<P>> o;
    win_expire_time(sp, I, now, o);
    emit(o);
  }
}

}  // namespace sg
