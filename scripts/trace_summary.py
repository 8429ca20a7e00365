"""Timeline of every traced span inside the bench's timed region (``RAYDP_TRACE=<prefix>``).

  RAYDP_TRACE=gpurun_out/tr/nyc python bench.py --steps 20 --warmup 5 --no-reference-config
  python scripts/trace_summary.py gpurun_out/tr/nyc > profiles/<name>.txt

Prints one line per span that starts inside the last ``timed run`` span (of the workload named
by the optional second argument): start offset and
duration in ms, the process, and the span name, indented by nesting within its process.
"""
import glob
import json
import sys


def main(prefix, workload=None):
    events = []
    for fn in sorted(glob.glob(f"{glob.escape(prefix)}.*.jsonl")):
        with open(fn) as f:
            for line in f:
                try:
                    e = json.loads(line)
                except ValueError:
                    continue
                if e.get("ph") == "X":
                    events.append(e)
                elif e.get("ph") == "i":
                    events.append(dict(e, dur=0.0))
    runs = [e for e in events if e["name"] == "timed run"
            and (workload is None or (e.get("args") or {}).get("workload") == workload)]
    if not runs:
        raise SystemExit("no 'timed run' span")
    run = runs[-1]
    t0, t1 = run["ts"], run["ts"] + run["dur"]
    inside = sorted((e for e in events if t0 <= e["ts"] <= t1), key=lambda e: (e["ts"], -e["dur"]))
    pname = {}
    print(f"timed run: {run['dur'] / 1000:.3f} ms")
    print(f"{'start':>8} {'dur':>8}  process  span")
    stack = {}
    for e in inside:
        pid = e["pid"]
        pname.setdefault(pid, e.get("cat", ""))
        st = [x for x in stack.get(pid, []) if x > e["ts"]]
        depth = len(st)
        st.append(e["ts"] + e["dur"])
        stack[pid] = st
        args = {k: v for k, v in (e.get("args") or {}).items()}
        extra = (" " + json.dumps(args)) if args else ""
        print(f"{(e['ts'] - t0) / 1000:8.3f} {e['dur'] / 1000:8.3f}  {pname[pid]:<8} {'  ' * depth}{e['name']}{extra}")


if __name__ == "__main__":
    # optional second argument: the workload whose timed run to show (default: the last one)
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
