"""Node-path probe on the GPU box: bench.py's C2 workload written to DIR, then
tools/bench_node.js at several round counts, one of them under node --cpu-prof
(the JS host's hot functions).  Usage: python tools/node_probe.py OUTDIR"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out = sys.argv[1]
    os.makedirs(out, exist_ok=True)
    import hashlib

    from bench import make_workload
    from lodestar_amd.native import Device
    dev = Device(0)
    sks, pks, msgs, sigs = make_workload(dev, 65536, 0, hashlib.sha256(b"lodestar-mi355x-bench").digest())
    dev.close()
    d = os.path.join(out, "data")
    os.makedirs(d, exist_ok=True)
    for name, items in (("pks", pks), ("msgs", msgs), ("sigs", sigs)):
        with open(os.path.join(d, name + ".bin"), "wb") as f:
            f.write(b"".join(items))
    res = {}
    # LB_PROBE_PREFETCH="0,1,2": one run per JS prefetch depth (packages packed ahead per GPU)
    variants = [int(x) for x in os.environ.get("LB_PROBE_PREFETCH", "0").split(",")]
    rounds_n = int(os.environ.get("LB_PROBE_ROUNDS", "96"))
    for pf in variants:
        env = dict(os.environ, LB_NODE_PRE="1", LB_JS_TRACE="1", LB_HOST_TRACE="1", LB_JS_PREFETCH=str(pf))
        rounds, prof = rounds_n, False
        cmd = ["node"] + (["--cpu-prof", "--cpu-prof-dir=" + os.path.join(out, "cpuprof")] if prof else []) + \
              [os.path.join(ROOT, "tools", "bench_node.js"), d, str(rounds)]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
        key = "rounds%d_prefetch%d%s" % (rounds, pf, "_prof" if prof else "")
        with open(os.path.join(out, key + "_stderr.txt"), "w") as f:
            f.write(r.stderr)
        ph = {}
        for line in r.stderr.splitlines():
            if line.startswith("lb_host_trace") and "sets=65536" in line:
                for kv in line.split()[2:]:
                    k, v = kv.split("=")
                    ph.setdefault(k, []).append(float(v))
        if ph:
            import statistics
            print(key, "host phases ms (mean / median):",
                  {k: (round(statistics.mean(v), 3), round(statistics.median(v), 3)) for k, v in ph.items()}, flush=True)
        res[key] = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else {"error": r.stderr[-800:]}
        print(key, json.dumps(res[key]), flush=True)
    with open(os.path.join(out, "node_probe.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
