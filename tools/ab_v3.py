"""A/B of two sweep builds on one box: python tools/ab_v3.py LIB_A LIB_B [rounds]
Runs bench.py (config 3, 10 steps) alternately with AME_LIB_PATH=A / B."""
import json, os, subprocess, sys
a, b = sys.argv[1], sys.argv[2]
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
res = {a: [], b: []}
for r in range(rounds):
    for lib in (a, b):
        env = dict(os.environ, AME_LIB_PATH=lib)
        out = subprocess.run([sys.executable, "-u", "bench.py", "--no-cpu-baseline", "--steps", "10", "--warmup", "3"],
                             env=env, capture_output=True, text=True, timeout=300)
        if out.returncode != 0:
            print(out.stderr[-2000:]); sys.exit(1)
        ms = json.loads(out.stdout.strip().splitlines()[-1])["ms_per_step"]
        res[lib].append(ms)
        print(os.path.basename(lib), round(ms, 4), flush=True)
for lib, v in res.items():
    print(os.path.basename(lib), "median", sorted(v)[len(v) // 2], v)
