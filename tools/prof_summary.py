"""Condense one rocprofv3 round (kernel trace + separate PMC passes) into a
committed summary under profiles/ (diagnostic tool, not the product).

Usage: python tools/prof_summary.py <prof_dir> <out_stem>

<prof_dir> is what tools/prof_round.sh wrote (kt/ and pmc_*/ subdirectories).
Writes <out_stem>.json (per engine kernel: calls, average duration, PMC
counters per dispatch, HBM traffic per dispatch) and <out_stem>_kernel_stats.csv
(the rocprofv3 --stats table restricted to the engine's kernels + torch's top
kernels).

HBM traffic per dispatch = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes): on gfx950
FETCH_SIZE counts half the bytes of wide streaming reads (MI355X_MICROARCH.md
section "HBM [CDNA4]"), WRITE_SIZE counts 16-B stores exactly.
"""

from __future__ import annotations

import csv
import json
import re
import sys
from collections import defaultdict
from pathlib import Path


# PIXEL pass A (the engine's 'pixel' timing bucket); the keyed wavelength
# coordinate pass ('coord' bucket on the sieve path)
COMPOSITES = {
    'pix_pass_a': ['k_pix_chunks', 'k_pix_count', 'k_pix_scan_blocks', 'k_pix_scan', 'k_pix_scatter'],
    'coord_keyed': ['k_key_dist', 'k_key_records', 'k_event_key'],
}


def short(name: str) -> str:
    m = re.search(r'lde::(k_\w+)', name)
    return m.group(1) if m else name.split('(')[0][:80]


def main(prof: Path, stem: Path) -> None:
    stats = list(csv.DictReader(open(prof / 'kt' / 'run_kernel_stats.csv')))
    kernels: dict[str, dict] = {}
    for r in stats:
        k = short(r['Name'])
        d = kernels.setdefault(k, {'calls': 0, 'total_ns': 0.0})
        d['calls'] += int(r['Calls'])
        d['total_ns'] += float(r['TotalDurationNs'])
    for d in kernels.values():
        d['avg_ms'] = d['total_ns'] / max(d['calls'], 1) / 1e6
    # steady-state average from the per-dispatch trace: every dispatch but a
    # kernel's first two (the bench's warm-up steps: first-touch allocations,
    # hot-set selection), comparable with the bench's timed-region stamps
    durs: dict[str, list[float]] = defaultdict(list)
    # and the idle time before each dispatch (previous dispatch's end to its
    # start): under tracing the dispatch lags the HIP start marker enqueued
    # ahead of it by about this much (the bench's event span includes it)
    gaps: dict[str, list[float]] = defaultdict(list)
    trace = prof / 'kt' / 'run_kernel_trace.csv'
    if trace.exists():
        rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r['Start_Timestamp']))
        prev_end = None
        for r in rows:
            s0, e0 = int(r['Start_Timestamp']), int(r['End_Timestamp'])
            k = short(r['Kernel_Name'])
            durs[k].append((e0 - s0) / 1e6)
            gaps[k].append(max(0, s0 - prev_end) / 1e6 if prev_end is not None else 0.0)
            prev_end = e0 if prev_end is None else max(prev_end, e0)
    counters: dict[str, dict[str, list[float]]] = defaultdict(lambda: defaultdict(list))
    for sub in sorted(prof.glob('pmc_*')):
        f = sub / 'run_counter_collection.csv'
        if not f.exists():
            continue
        per = defaultdict(float)  # (kernel, dispatch, counter) -> value summed over dims
        for r in csv.DictReader(open(f)):
            per[(short(r['Kernel_Name']), r['Dispatch_Id'], r['Counter_Name'])] += float(r['Counter_Value'])
        for (k, _, c), v in per.items():
            counters[k][c].append(v)
    out = {}
    for k, d in kernels.items():
        if not k.startswith('k_'):
            continue
        e = {'calls': d['calls'], 'avg_ms': d['avg_ms']}
        if len(durs.get(k, [])) > 2:
            # past the first two, the dispatches of the bench's step batch:
            # launches under half the median are other sizes (the wavelength
            # bench's parity check bins a smaller batch after the timed steps)
            st = durs[k][2:]
            med = sorted(st)[len(st) // 2]
            st = [x for x in st if x >= 0.5 * med]
            e['avg_ms_steady'] = sum(st) / len(st)
            g = sorted(gaps[k][2:])  # median: the steps after the timed region wait on the host
            e['gap_before_ms_steady'] = g[len(g) // 2]
        pm = {c: sum(v) / len(v) for c, v in counters.get(k, {}).items()}
        # the first dispatches of each kernel include warm-up sizes; use the median-like mean
        e['pmc_per_dispatch'] = pm
        if 'FETCH_SIZE' in pm and 'WRITE_SIZE' in pm:
            e['hbm_read_bytes'] = 2 * pm['FETCH_SIZE'] * 1024
            e['hbm_write_bytes'] = pm['WRITE_SIZE'] * 1024
            e['hbm_traffic_bytes'] = e['hbm_read_bytes'] + e['hbm_write_bytes']
            e['hbm_GBs_at_avg'] = e['hbm_traffic_bytes'] / (d['avg_ms'] * 1e-3) / 1e9
        out[k] = e
    # composite entries for engine timing buckets that span several launches:
    # per launch of the last member (launched once per batch), the members'
    # time and traffic per dispatch weighted by their launches per batch (a
    # PIXEL batch with predicted slots has no k_pix_count: only the counted
    # first batch does)
    for name, members in COMPOSITES.items():
        names = [m for m in members if m in out]
        ms = [out[m] for m in names]
        if not ms or members[-1] not in out:
            continue
        n = out[members[-1]]['calls']
        w = [m['calls'] / n for m in ms]
        e = {'members': names, 'calls': n,
             'launches_per_call': {m: round(x, 4) for m, x in zip(names, w)},
             'avg_ms': sum(x * m['avg_ms'] for x, m in zip(w, ms))}
        # steady state: past each member's first two dispatches; a member
        # launched only in the warm-up steps (k_pix_count: the first,
        # counted batch) is not part of the steady step
        n_last = len(durs.get(members[-1], []))
        if n_last > 2:
            e['avg_ms_steady'] = sum(sum(durs[m][2:]) for m in names) / (n_last - 2)
        if all('hbm_traffic_bytes' in m for m in ms):
            for key in ('hbm_read_bytes', 'hbm_write_bytes', 'hbm_traffic_bytes'):
                e[key] = sum(x * m[key] for x, m in zip(w, ms))
            e['hbm_GBs_at_avg'] = e['hbm_traffic_bytes'] / (e['avg_ms'] * 1e-3) / 1e9
        out[name] = e
    stem.parent.mkdir(parents=True, exist_ok=True)
    Path(str(stem) + '.json').write_text(json.dumps(out, indent=1, sort_keys=True) + '\n')
    rows = sorted(stats, key=lambda r: -float(r['TotalDurationNs']))
    with open(str(stem) + '_kernel_stats.csv', 'w', newline='') as f:
        w = csv.writer(f)
        w.writerow(['Name', 'Calls', 'TotalDurationNs', 'AverageNs', 'Percentage', 'MinNs', 'MaxNs'])
        for r in rows:
            if 'lde::' in r['Name'] or rows.index(r) < 8:
                w.writerow([short(r['Name']), r['Calls'], r['TotalDurationNs'], r['AverageNs'],
                            r['Percentage'], r['MinNs'], r['MaxNs']])
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == '__main__':
    main(Path(sys.argv[1]), Path(sys.argv[2]))
