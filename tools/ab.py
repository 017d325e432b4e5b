"""A/B decode variants in separate processes (env vars select kernel variants), interleaved
rounds to cancel box drift.  Usage: python tools/ab.py 'NAME=ENV=VAL,ENV=VAL' ... [--rounds R]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
args = [a for a in sys.argv[1:] if not a.startswith("--")]
rounds = 3
for a in sys.argv[1:]:
    if a.startswith("--rounds="):
        rounds = int(a.split("=")[1])
variants = []
for a in args:
    name, _, envs = a.partition("=")
    env = dict(os.environ)
    for kv in filter(None, envs.split(",")):
        k, _, v = kv.partition("=")
        env[k] = v
    variants.append((name, env))
res = {name: [] for name, _ in variants}
for _ in range(rounds):
    for name, env in variants:
        out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "bench_variants.py"), "jit"],
                             env=env, capture_output=True, text=True, timeout=300)
        if out.returncode != 0:
            print(out.stderr[-2000:])
            sys.exit(1)
        d = json.loads(out.stdout.strip().splitlines()[-1])
        res[name].append(d["jit"]["med"])
summary = {k: {"median_ms": sorted(v)[len(v) // 2], "all": v} for k, v in res.items()}
print(json.dumps(summary))
