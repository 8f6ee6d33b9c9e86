#!/usr/bin/env python3
"""Print compact summaries of gpurun_out/ artefacts: bench JSON lines, microbench tables, pytest tails.
Usage: python tools/summarize.py gpurun_out/bench*.log gpurun_out/kbench.log gpurun_out/pytest_gpu.log"""
import collections
import json
import sys


def main(paths):
    kb = collections.defaultdict(dict)
    for p in paths:
        try:
            lines = open(p).read().strip().split("\n")
        except OSError as e:
            print(p, "missing", e)
            continue
        if "pytest" in p:
            print(p, "|", lines[-1])
            continue
        for ln in lines:
            if not ln.startswith("{"):
                continue
            r = json.loads(ln)
            if "metric" in r:
                print(f"{p}: B={r['config']['global_batch']} {r['value']} tok/s, decode {r['decode_ms_per_token']} ms/tok, "
                      f"ttft {r['ttft_ms']} ms, step {r['ms_per_step']} ms")
            elif "variant" in r:
                kb[(r["op"], r["m"])][r["variant"]] = r["us"]
            else:
                print(p, r)
    for k, v in kb.items():
        print(k, v)


if __name__ == "__main__":
    main(sys.argv[1:])
