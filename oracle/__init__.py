"""ORACLE — test infrastructure only, never shipped, never on the product path.

This package is a CPU restatement (numpy for the index/byte ops, torch fp32 CPU for
the floating-point ops) of the Swin + Mask2Former training hot path that
`BASELINE.json`'s north star names.  The reference repository
(Wlsghdh/VISION-Instance-Seg) contains no implementation of that path:
it drives upstream MaskDINO / Mask2Former through detectron2, neither of which is in
this container.  The arithmetic therefore follows the in-container third-party
implementation that SURVEY §8(c) designates as the oracle:

    transformers 5.15.0 (pinned: the version installed in the build container)
      HF:swin = transformers/models/swin/modeling_swin.py
      HF:m2f  = transformers/models/mask2former/modeling_mask2former.py

Every function cites the HF file:line it restates.  The restatement is *pinned* by
golden vectors generated from HF itself in the build container
(`tests/golden/gen_golden.py` -> `tests/golden/*.npz`); `tests/test_oracle_golden.py`
checks it against them (index ops bit-exact, float ops <= 1e-5 fp32).  MaskDINO-only
parts (config C4) have no in-container implementation: parity unpinned there.

Who may import this package: `tests/`, `__graft_entry__.smoke()` and the
`cpu_baseline` leg of `bench.py` — as the checker / timed CPU baseline only.
"""
