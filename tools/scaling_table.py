"""Turn bench JSON lines (the driver's SCALE_r*.json, BENCH_r*.json, or bench.py output) into the
report's Tables 1-3 layout: time, speedup and efficiency per GPU count (Report.pdf p.21-22).

  python tools/scaling_table.py SCALE_r02.json [more.json ...]
Speedup here is T(1 GPU)/T(N GPUs) of the same grid from the same file set (strong scaling) or
value_N / (N * value_1) as efficiency (weak scaling); each row also shows the in-job speedup the
bench itself measured when present.
"""
import json
import sys


def records(path):
    txt = open(path).read()
    try:
        d = json.loads(txt)
        cands = [d]
    except json.JSONDecodeError:
        cands = [json.loads(l) for l in txt.splitlines() if l.strip().startswith("{")]
    out = []
    for d in cands:
        if isinstance(d, dict) and "runs" in d and isinstance(d["runs"], (list, dict)):  # driver SCALE layout
            runs = d["runs"].values() if isinstance(d["runs"], dict) else d["runs"]
            for r in runs:
                p = r.get("parsed") if isinstance(r, dict) else None
                if p:
                    out.append(p)
        elif isinstance(d, dict) and "parsed" in d:
            out.append(d["parsed"])
        elif isinstance(d, dict) and "value" in d:
            out.append(d)
    return out


def table(recs):
    recs = sorted(recs, key=lambda r: r["n_gpus"])
    base = next((r for r in recs if r["n_gpus"] == 1), None)
    print(f"{'GPUs':>4} {'grid':>14} {'ms/step':>9} {'cell-updates/s':>15} {'speedup':>8} {'eff.':>6} "
          f"{'in-job S':>8} {'in-job E':>8} {'halo wait':>9}  transport/pipeline")
    for r in recs:
        g = r.get("config", {}).get("grid", ["?", "?"])
        if base:
            if r.get("scaling") == "weak":
                e = r["value"] / (r["n_gpus"] * base["value"])
                s = e * r["n_gpus"]
            else:
                s = r["value"] / base["value"]
                e = s / r["n_gpus"]
        else:
            s = e = float("nan")
        js, je = r.get("speedup"), r.get("efficiency")
        tp = f"{r.get('config', {}).get('transport', '')}/{r.get('config', {}).get('pipeline', '')}"
        # exposed halo wait as a share of a chunk (the reference's MPI_Waitall share, Report p.34-37)
        hw = (r.get("halo_wait") or {}).get("share_of_chunk")
        hws = f"{100 * hw:8.1f}%" if hw is not None else f"{'-':>9}"
        print(f"{r['n_gpus']:>4} {str(g[0]) + 'x' + str(g[1]):>14} {r['ms_per_step']:9.4f} {r['value']:15.4e} "
              f"{s:8.2f} {e:6.2f} {js if js is not None else float('nan'):8.2f} "
              f"{je if je is not None else float('nan'):8.2f} {hws}  {tp}")


if __name__ == "__main__":
    allr = []
    for p in sys.argv[1:]:
        allr += records(p)
    if not allr:
        sys.exit("no bench records found")
    table(allr)
