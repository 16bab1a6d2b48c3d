"""Probe: bench.py's drop-in legs alone (time_api: the inference.py loop through the drop-in module, with and
without the lookahead, then the ablation harness), repeated, to separate a box's noise from a change.
    python tools/probes/api_probe.py [--rounds 2] [--tokens 32]"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--tokens", type=int, default=32)
    a = ap.parse_args()
    from pgmi.synthetic import paligemma_3b_config
    cfg = paligemma_3b_config(224)
    dev = torch.device("cuda", 0)
    for r in range(a.rounds):
        res = bench.time_api(cfg, dev, 1234, a.tokens)
        h = res["ablation_harness"]
        print(f"round {r}: drop-in {res['decode_ms_per_token']} ms/token (no lookahead "
              f"{res['decode_ms_per_token_no_lookahead']}), harness {h['steady_ms_per_token']} ms/token", flush=True)


if __name__ == "__main__":
    main()
