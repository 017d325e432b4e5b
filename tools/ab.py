"""A/B kernel variants in separate processes (env vars select kernel variants), interleaved
rounds to cancel box drift.
Usage: python tools/ab.py 'NAME=ENV=VAL,ENV=VAL' ... [--rounds=R] [--tool=flat|nested]
  flat:   tools/bench_variants.py jit  (1M Flat16 decode, median per-launch ms)
  nested: tools/bench_nested.py        (1M Nested one-pass decode, ms per launch)
  encode / nested_encode: tools/bench_encode.py (flat / nested encode ms)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
args = [a for a in sys.argv[1:] if not a.startswith("--")]
rounds, tool = 3, "flat"
for a in sys.argv[1:]:
    if a.startswith("--rounds="):
        rounds = int(a.split("=")[1])
    if a.startswith("--tool="):
        tool = a.split("=")[1]
cmd, key = {"flat": (["bench_variants.py", "jit"], "jit"), "nested": (["bench_nested.py"], "nested"),
            "encode": (["bench_encode.py"], "flat"), "nested_encode": (["bench_encode.py", "nested"], "nested")}[tool]
field = "encode_ms" if tool == "nested_encode" else "med"
variants = []
for a in args:
    name, _, envs = a.partition("=")
    env = dict(os.environ)
    for kv in filter(None, envs.split(",")):
        k, _, v = kv.partition("=")
        env[k] = v
    variants.append((name, env))
res = {name: [] for name, _ in variants}
extra = {}
for _ in range(rounds):
    for name, env in variants:
        out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", cmd[0])] + cmd[1:],
                             env=env, capture_output=True, text=True, timeout=300)
        if out.returncode != 0:
            print(out.stderr[-2000:])
            sys.exit(1)
        d = json.loads(out.stdout.strip().splitlines()[-1])
        res[name].append(d[key][field])
        extra[name] = d[key]
summary = {k: {"median_ms": sorted(v)[len(v) // 2], "all": v, "last": extra[k]} for k, v in res.items()}
print(json.dumps(summary))
