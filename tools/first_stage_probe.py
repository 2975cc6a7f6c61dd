"""Why does a pipeline's first stage run its layers ~3.5 % slower than the others?
(profiles/r05/stage_projection_sublayer.json: stage 0's measured / predicted ratio is ~1.00,
every other stage's ~0.97.)  Times the same 5-layer range (bench.stage_ms, B = 16, ctx 2048)
as a first stage (embedding, token ids) and as an inner stage fed hidden states of three
scales -- randn x 0.5 (bench.stage_ms's inner-stage input), randn x 0.035 (the embedding's
scale) and the embedding rows themselves -- twice each, interleaved.

  python tools/first_stage_probe.py > gpurun_out/first_stage_probe.json
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from inferd_amd.pipeline import StageRange  # noqa: E402
from inferd_amd.runtime import GLOBAL_TENSOR_IDS, MODELS, gen_tensor  # noqa: E402


def main():
    d = MODELS["qwen3-8b"]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B, ctx, seed = 16, 2048, 1234
    r = StageRange(0, 10)
    emb = gen_tensor(seed, GLOBAL_TENSOR_IDS["embed_tokens"], (d.vocab, d.hidden), False, dev)
    t0 = time.time()
    res = {}
    orig_randn = torch.randn

    def run(tag, first, scale=None, embed=False, ballast=None):
        g = torch.Generator(device="cpu").manual_seed(5)
        hold = None
        if ballast == "before":   # 1.24 GB allocated before the span (the embedding table's size)
            hold = torch.empty(d.vocab * d.hidden, dtype=torch.bfloat16, device=dev)
        if embed:     # inner stage fed embedding rows (what stage 0's layers see)
            def fake(*shape, generator=None, **kw):
                n = 1
                for s in shape:
                    n *= s
                ids = torch.randint(0, d.vocab, (n // d.hidden,), generator=generator)
                return emb[ids.to(dev)].float().cpu().reshape(shape) / 0.5
            torch.randn = fake
        elif scale is not None:
            torch.randn = lambda *a, **k: orig_randn(*a, **k) * (scale / 0.5)
        try:
            ms = bench.stage_ms(d, r, first, False, B, ctx, dev, g, seed, warmup=5, reps=40)
        finally:
            torch.randn = orig_randn
        del hold
        res.setdefault(tag, []).append(round(ms * 1e3, 2))
        print(f"[{time.time() - t0:6.1f}s] {tag}: {ms * 1e3:.1f} us", file=sys.stderr, flush=True)

    only = sys.argv[1] if len(sys.argv) > 1 else ""    # "first" / "inner" / "ballast": one kind
    for _ in range(2):
        if only in ("", "first"):
            run("first_ids", True)
        if only in ("", "inner"):
            run("inner_randn0.5", False)
        if not only:
            run("inner_randn0.035", False, scale=0.035)
            run("inner_embed_rows", False, embed=True)
        if only in ("", "ballast"):
            run("inner_ballast_before", False, ballast="before")
            run("inner_plain", False)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
