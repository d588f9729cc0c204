// Zero-copy policy: the schedule an allreduce runs once registered buffers (flexar_reg_*) are in play.
// A pure function of the call's resolved spec and a few facts about the call, so comm.hip applies it on
// the hot path and tests/test_zero_copy.py checks it on the CPU (flexar_zc_decide).
//  * registered buffers + a choice the call did not name (cost model or tune table; communicator default
//    "auto"): the flat schedule switches to "+zc+push" (no staging); another model choice (oneshot, LL,
//    ring, trees) switches when the cost model prices the zero-copy push form lower - a tune table's
//    measured non-flat choice is kept; never when the zero-copy form's protocol family failed the
//    connect-time self-test
//  * a zero-copy choice the call did not name (tune table, default spec) on unregistered buffers falls
//    back to the staging flat schedule; an explicit "+zc" on unregistered buffers stays an error (zc_bind)
// Registration is collective, so every rank reaches the same decision.
#pragma once

#include <stdint.h>

#include "flexar/cost_model.hpp"
#include "flexar/readiness.hpp"

namespace flexar {

struct ZcFacts {
  int nranks = 1;
  double bytes = 0;
  bool registered = false;  // both buffers of the call lie inside registrations
  bool named = false;       // the call named a spec (not NULL / "auto")
  bool from_auto = false;   // neither the call nor the communicator default named one
  bool zc_auto = true;      // FLEXAR_ZC_AUTO
  bool have_tune = false;   // a measured tune table is installed
  uint32_t disabled = 0;    // protocol families that failed the connect-time self-test
  uint32_t esize = 4;       // element size the cost model prices the two forms at
};

// Returns 1 when the spec switched to zero copy, -1 when it fell back to staging, 0 when unchanged.
inline int zc_decide(AlgoSpec* s, const ZcFacts& f, const XgmiModel& m) {
  const bool flat = s->kind == AlgoKind::TREE && s->widths.size() == 1 && !s->msg && s->wire == 0 && f.nranks > 1;
  const bool reg = f.registered && f.nranks > 1 && !s->msg && s->wire == 0;
  if (reg && !s->zc && f.from_auto && f.zc_auto && s->kind != AlgoKind::DMA) {
    AlgoSpec z;
    z.kind = AlgoKind::TREE;
    z.widths = {f.nranks};
    z.ag = AgMode::PUSH;
    z.zc = true;
    z.wt = s->wt;
    z.nts = s->nts;
    if (f.disabled & proto_family(z)) return 0;
    if (flat || (!f.have_tune && m.cost_us(z, f.nranks, f.bytes, f.esize) < m.cost_us(*s, f.nranks, f.bytes, f.esize))) {
      *s = z;
      return 1;
    }
    return 0;
  }
  if (flat && s->zc && !f.registered && !f.named) {
    s->zc = false;
    s->put = false;
    return -1;
  }
  return 0;
}

}  // namespace flexar
