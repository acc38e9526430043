"""A/B tooling only: translate the experiment environment of the older scripts
(MI355X_GEMV_PRE0=3 python ... etc.) into explicit library calls. The product
library reads no environment (tests/test_abi.py); tools call apply_env() at start.

  MI355X_<KNOB>=v          -> ggml_mi355x.debug_knob("<KNOB>", v)   (DEBUG_KNOBS)
  MI355X_GEMV_IMPL=tasks|rows, MI355X_MMQ_IMPL=tile64|..., MI355X_PREFILL=f16|f16_all,
  MI355X_ATTN_IMPL=group|head|split -> the matching selector call
"""
import os

import ggml_mi355x as g


def apply_env(environ=None):
    env = os.environ if environ is None else environ
    done = {}
    for k in g.DEBUG_KNOBS:
        v = env.get("MI355X_" + k)
        if v is not None:
            g.debug_knob(k, float(v))
            done[k] = float(v)
    sel = {
        "MI355X_GEMV_IMPL": (g.gemv_impl, {"tasks": g.GEMV_TASKS, "rows": g.GEMV_ROWS, "auto": g.GEMV_AUTO,
                                           "dyn": g.GEMV_DYN}),
        "MI355X_MMQ_IMPL": (g.mmq_impl, {"tile64": g.MMQ_TILE64, "tile128": g.MMQ_TILE128,
                                         "tile128w": g.MMQ_TILE128W, "tile64w": g.MMQ_TILE64W, "tile128x": g.MMQ_TILE128X, "tile192": g.MMQ_TILE192,
                                         "auto": g.MMQ_AUTO}),
        "MI355X_PREFILL": (g.prefill_precision, {"f16": g.PREFILL_F16, "f16_all": g.PREFILL_F16_ALL,
                                                 "exact": g.PREFILL_EXACT}),
        "MI355X_ATTN_IMPL": (g.attn_impl, {"group": g.ATTN_GROUP, "head": g.ATTN_HEAD, "split": g.ATTN_SPLIT}),
    }
    for name, (fn, table) in sel.items():
        v = env.get(name)
        if v is not None:
            fn(table[v])
            done[name] = v
    return done
