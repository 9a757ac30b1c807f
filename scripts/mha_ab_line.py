"""Compact one line of scripts/bench_mha.py output: kernel -> avg_ms (used by gpu_mha_ab.sh)."""
import json
import sys

for line in open(sys.argv[1]):
    line = line.strip()
    if line.startswith("{"):
        d = json.loads(line)
        print(" ".join(f"{k.replace('_mha', '')}={v['avg_ms']}" for k, v in d.items()))
