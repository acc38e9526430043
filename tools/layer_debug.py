"""Debug aid for the persistent decode layer: one small decoder (tests/test_gpu_layer.py's
TinyLlama shape, a chosen mix), engine on vs off, eager and graph, printing per-token
logits agreement and simple statistics.
    python tools/layer_debug.py [--mix q5_k_m] [--tokens 3]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ggml-neon-opt_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mix", default="q5_k_m")
    ap.add_argument("--tokens", type=int, default=3)
    ap.add_argument("--shape", default="2048,2,32,4,5632,4096")
    args = ap.parse_args()
    from tests import llama_model as LM
    import ggml_mi355x as g
    from ggml_mi355x.llama import LlamaDecoder, hparams
    dev = torch.device("cuda:0")
    hp = hparams(*[int(v) for v in args.shape.split(",")])
    w = LM.build(hp, 31, mix=args.mix)
    wd = LM.to_device(w, dev)
    toks = np.random.default_rng(5).integers(0, hp["n_vocab"], size=args.tokens).tolist()
    res = {}
    for eng in (False, True):
        for graph in (False, True):
            b = g.Backend()
            b.set_layer_engine(eng)
            dec = LlamaDecoder(b, hp, wd, 64, fuse=True)
            outs = []
            for p, t in enumerate(toks):
                dec.step(t, p, use_graph=graph)
                b.synchronize()
                outs.append((dec.logits.cpu().numpy().copy(), dec.last_hidden.cpu().numpy().copy()))
            res[(eng, graph)] = outs
            print(f"engine={eng} graph={graph} layer_error={b.layer_error()}", flush=True)
            b.close()
    base = res[(False, False)]
    for k, outs in res.items():
        for p, (lg, hd) in enumerate(outs):
            same = np.array_equal(lg.view(np.uint32), base[p][0].view(np.uint32))
            print(k, p, "same" if same else "DIFF", "zeros", int((lg == 0).sum()), "nan", int(np.isnan(lg).sum()),
                  "hid absmax", float(np.abs(hd).max()), "hid zeros", int((hd == 0).sum()), flush=True)


if __name__ == "__main__":
    main()
