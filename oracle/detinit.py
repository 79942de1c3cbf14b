"""ORACLE (test infrastructure only) — deterministic weights for parity runs.

Golden fixtures do not store model weights: both the fixture generator (which loads
them into the HF oracle) and the tests (which load them into the oracle restatement
and into the GPU build) regenerate them from a seed with this function, so the
fixtures stay small.  Plain `torch.randn` on a CPU generator, parameters visited in
sorted-name order: identical on every machine running the same torch build.
"""
from __future__ import annotations

import math

import torch


def det_init(shapes: dict, seed: int = 1234) -> dict:
    """shapes: {name: torch.Size} in the build layout -> {name: fp32 CPU tensor}."""
    g = torch.Generator().manual_seed(seed)
    out = {}
    for name in sorted(shapes):
        shp = tuple(shapes[name])
        r = torch.randn(shp, generator=g, dtype=torch.float32)
        leaf = name.rsplit(".", 1)[-1]
        is_norm = any(t in name for t in ("norm", ".gn.")) and leaf in ("weight", "bias")
        if is_norm and leaf == "weight":
            t = 1.0 + 0.1 * r
        elif leaf == "bias" and "sampling_offsets" in name:
            t = 1.5 * r                      # offsets of a few pixels, all directions
        elif leaf == "bias":
            t = 0.05 * r
        elif "rel_table" in name:
            t = 0.5 * r
        elif "level_embed" in name or "query_" in name:
            t = 0.5 * r
        elif "sampling_offsets" in name or "attention_weights.weight" in name:
            t = r * (0.5 / math.sqrt(shp[-1]))
        elif len(shp) >= 2:
            fan_in = int(torch.tensor(shp[1:]).prod())
            t = r / math.sqrt(fan_in)
        else:
            t = 0.1 * r
        out[name] = t.contiguous()
    return out
