"""A/B of sweep builds on one box: python tools/ab_v3.py LIB_A LIB_B [LIB_C ...] [--rounds N] [-- bench args]
Runs bench.py (config 3, 10 steps by default) round-robin with AME_LIB_PATH set to each library."""
import json, os, subprocess, sys

args = sys.argv[1:]
extra = []
if "--" in args:
    k = args.index("--")
    args, extra = args[:k], args[k + 1:]
rounds = 3
if "--rounds" in args:
    k = args.index("--rounds")
    rounds = int(args[k + 1])
    del args[k:k + 2]
libs = args
bench = extra or ["--steps", "10", "--warmup", "3"]
res = {lib: [] for lib in libs}
for r in range(rounds):
    for lib in libs:
        env = dict(os.environ, AME_LIB_PATH=lib)
        out = subprocess.run([sys.executable, "-u", "bench.py", "--no-cpu-baseline", *bench],
                             env=env, capture_output=True, text=True, timeout=300)
        if out.returncode != 0:
            print(out.stderr[-2000:]); sys.exit(1)
        ms = json.loads(out.stdout.strip().splitlines()[-1])["ms_per_step"]
        res[lib].append(ms)
        print(os.path.basename(lib), round(ms, 4), flush=True)
for lib, v in res.items():
    print(os.path.basename(lib), "median", round(sorted(v)[len(v) // 2], 4), [round(x, 4) for x in v])
