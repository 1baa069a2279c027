"""Node-path probe (round 5): bench.py's C2 workload and C4 aggregates written to a
directory, then tools/bench_node.js with the JS host's per-call trace (LB_JS_TRACE=1)
and V8's GC log (--trace-gc), to find where a lone call's time goes after the
throughput phase and under load.  Usage: python tools/node_probe_r05.py OUTDIR [ROUNDS]"""
import hashlib
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def write_data(d):
    from bench import compress_g1, make_workload
    from lodestar_amd.native import Device
    dev = Device(0)
    sks, pks, msgs, sigs = make_workload(dev, 65536, 0, hashlib.sha256(b"lodestar-mi355x-bench").digest())
    dev.close()
    for name, items in (("pks", pks), ("msgs", msgs), ("sigs", sigs)):
        with open(os.path.join(d, name + ".bin"), "wb") as f:
            f.write(b"".join(items))
    with open(os.path.join(d, "pks_c.bin"), "wb") as f:
        f.write(b"".join(compress_g1(k) for k in pks))


def main():
    if sys.argv[1] == "--write-data":
        write_data(sys.argv[2])
        return
    out = sys.argv[1]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 96
    os.makedirs(out, exist_ok=True)
    import tempfile
    d = tempfile.mkdtemp(prefix="lb_node_probe_")  # (not under gpurun_out: ~17 MB of inputs)
    if os.environ.get("LB_PROBE_CHILD_DATA") == "1":
        # the inputs from a child process: this one never opens a HIP queue (HIP may keep
        # a process's hardware queues after its streams are destroyed)
        subprocess.run([sys.executable, os.path.abspath(__file__), "--write-data", d], check=True, timeout=300)
    else:
        write_data(d)
    env = dict(os.environ, LB_JS_TRACE="1")
    extra = os.environ.get("LB_NODE_FLAGS", "--trace-gc").split()
    r = subprocess.run(["node"] + extra + [os.path.join(ROOT, "tools", "bench_node.js"), d, str(rounds)],
                       capture_output=True, text=True, timeout=400, env=env)
    with open(os.path.join(out, "node_stdout.txt"), "w") as f:
        f.write(r.stdout)
    with open(os.path.join(out, "node_stderr.txt"), "w") as f:
        f.write(r.stderr)
    lines = r.stdout.strip().splitlines()
    gc = [ln for ln in lines if "Mark-sweep" in ln or "Scavenge" in ln or "Mark-Compact" in ln]
    pauses = [float(m.group(1)) for ln in gc for m in [re.search(r"([\d.]+) / [\d.]+ ms", ln)] if m]
    res = json.loads(lines[-1]) if lines and lines[-1].startswith("{") else {"rc": r.returncode, "err": r.stderr[-800:]}
    res["gc"] = {"events": len(gc), "pause_ms_total": round(sum(pauses), 1),
                 "pause_ms_max": round(max(pauses), 1) if pauses else 0,
                 "mark_sweep": sum(1 for ln in gc if "Mark" in ln)}
    import shutil
    shutil.rmtree(d, ignore_errors=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
