#!/usr/bin/env python
"""Benchmark: binned events/s for a DREAM-scale detector view on MI355X.

Workload (BASELINE.json configs[2], "DREAM cylinder_mantle_z projection with
noise replicas + TOA binning (non-uniform edges), skewed hot-pixel
distribution"): 491,520-pixel mantle, 80 x 320 screen, 5 replicas, 100
geomspace TOA bins, Zipf(1.2) pixel skew + 3 hot TOA bins.  One step = one 1 Hz
service batch: 14 ev44 pulses of 1e7 events each (1.4e8 events) staged from
HBM, binned into the current window (accumulate), then finalized (cumulative
+= window, images and totals to the host).  With N > 1 ranks every rank bins
its own batch (event-batch sharding, weak scaling) into its own histograms, and
each finalize RCCL-reduces the ranks' exact partial outputs (u64 images and
totals) onto rank 0 over xGMI.

Prints ONE JSON line on rank 0.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

PROFILE_ROUND = 'r6'  # profiles/<round>_<workload>_bench.json (tools/prof_round.sh)
# bench kernel name -> device symbol in the rocprofv3 summary
KERNEL_SYMBOL = {
    'atomic': 'k_bin_atomic',
    'partition': 'k_partition',
    'tile_accumulate': 'k_tile_accumulate',
    'paged': 'k_paged_partition',
    'page_accumulate': 'k_page_accumulate',  # (PIXEL's pass B, k_pix_accumulate, shares the bucket)
    'split': 'k_sieve',  # SPLIT's event pass
    'coord': 'k_event_key',  # wavelength-mode keyed coordinate pass (its per-replica tables cached)
    'pixel': 'k_pix_scatter',  # PIXEL pass A's partition kernel (after k_pix_chunks and the scans)
    'monitor': 'k_monitor',  # monitor TOA histogram (--workload monitor)
    'finalize': 'k_finalize_v4',
    'wide': 'k_wide_scatter',  # WIDE first pass (keys into page chains)
    'wide_accumulate': 'k_wide_accumulate',  # WIDE pass B (tiles in LDS)
}
# engine timing buckets (include/lde.h LDE_K_*) as they are used by the SPLIT
# strategy's SIEVE pass: 'split' = k_sieve, 'split_aux' = hot-set selection,
# 'paged' = the cold-key pipeline (k_hot_reduce_scan, k_cold_sort,
# k_cold_accumulate)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, spec)
BYTES_PER_EVENT = 8  # int32 pixel_id + int32 time_of_flight
# the wavelength-mode coordinate pass also writes its 4-byte per-event word
KERNEL_BYTES_PER_EVENT = {'coord': 12, 'monitor': 4}
MONITOR_BYTES_PER_EVENT = 4  # int32 time_of_arrival only


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--workload', default='dream', choices=['dream', 'loki', 'monitor', 'bifrost'],
                    help='monitor: the beam-monitor TOA histogram (A13), 1e7 events per pulse '
                         'into 100 bins; bifrost: 45 bank messages of 1,000 events per pulse into '
                         'the float32 15 x 900 unified view, one accumulate (f32 push) per pulse, '
                         'one finalize per step (diagnostic lines, not the headline metric)')
    ap.add_argument('--coordinate', default='toa', choices=['toa', 'wavelength'],
                    help='wavelength: DREAM events binned by wavelength through a direct-flight '
                         'lookup table (diagnostic line, not the headline metric)')
    ap.add_argument('--pulses', type=int, default=14)
    ap.add_argument('--events-per-pulse', type=int, default=10_000_000)
    ap.add_argument('--strategy', default='auto', choices=['auto', 'atomic', 'partition', 'paged', 'split', 'pixel', 'wide'])
    ap.add_argument('--view', default='geometric',
                    choices=['geometric', 'mantle_front_layer', 'wire_view', 'strip_view'],
                    help='DREAM logical views (dream/specs.py:151-180) instead of the '
                         'cylinder_mantle_z projection (diagnostic lines, not the headline)')
    ap.add_argument('--cpu-baseline-seconds', type=float, default=12.0)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-finalize-overlap', dest='finalize_overlap', action='store_false',
                    help='wait for each finalize before the next batch is enqueued (default: '
                         'the next batch is binned while the host reads the outputs)')
    ap.add_argument('--timing-stride', type=int, default=5,
                    help='stamp the dominant kernel with HIP events on every Nth timed step '
                         '(a stamped dispatch costs ~16 us of step time on the sieve path)')
    ap.add_argument('--e2e-steps', type=int, default=3,
                    help='steps of the PCIe-inclusive host-staged leg (0 = skip)')
    ap.add_argument('--batches', type=int, default=3,
                    help='distinct pre-generated batches rotated through the steps (a stream '
                         'never repeats the previous batch, so per-batch predictions are tested)')
    ap.add_argument('--bifrost-cadence', default='batch', choices=['batch', 'pulse'],
                    help='batch (the reference cadence, core/job.py:413-433): one accumulate of '
                         'all 14 x 45 bank messages (one float32 push) and one finalize per step; '
                         'pulse: one push per pulse, 14 per finalize')
    ap.add_argument('--shard', default='events', choices=['events', 'banks'],
                    help='events: every rank bins its own DREAM batches (event-batch sharding); '
                         "banks: LOKI's nine banks placed on the ranks by assign_banks, each rank "
                         "binning its banks' streams with no collective (pixel-range sharding)")
    ap.add_argument('--num-bins', type=int, default=None,
                    help='TOA bins of the detector view (EdgesModel.num_bins, 1..10000, '
                         'parameter_models.py:87); default: the instrument\'s (100)')
    ap.add_argument('--toa-scale', default=None, choices=['linear', 'log'],
                    help="TOA edge scale (default: the instrument's)")
    ap.add_argument('--toa-start', type=float, default=None,
                    help="first TOA edge in ms (default: the instrument's; log needs > 0)")
    ap.add_argument('--bank-steps', type=int, default=5,
                    help='timed steps of the bank-sharded LOKI leg reported beside the DREAM line '
                         '(bank_sharding; 0 = skip)')
    return ap.parse_args()


def launch_ranks(args) -> int:
    """``--gpus N`` (N > 1) without a torchrun environment: start N rank
    processes as children (``torch.distributed.run``, one rank per GPU,
    rendezvous on 127.0.0.1) and return their exit code.  This process never
    initialises HIP (``torch.cuda.device_count`` does not), so no process that
    touched the GPU is replaced; the ranks' stdout (rank 0's JSON line) passes
    through.  ``LDE_BENCH_BACKEND=gloo`` rehearses N ranks on fewer GPUs."""
    import socket
    import subprocess

    backend = os.environ.get('LDE_BENCH_BACKEND', 'nccl')
    if backend == 'nccl':
        import torch

        visible = torch.cuda.device_count()
        if args.gpus > visible:
            print(f'bench.py: --gpus {args.gpus} but {visible} GPU(s) visible '
                  '(LDE_BENCH_BACKEND=gloo rehearses ranks sharing a GPU)', file=sys.stderr)
            return 2
    with socket.socket() as s:  # a free rendezvous port on the loopback
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
           f'--nproc-per-node={args.gpus}', '--master-addr=127.0.0.1', f'--master-port={port}',
           str(ROOT / 'bench.py'), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault('OMP_NUM_THREADS', str(max(1, min(16, len(os.sched_getaffinity(0)) // args.gpus))))
    return subprocess.run(cmd, env=env).returncode


def cpu_baseline(inst, ps, view, pid_h, toa_h, replica, gpu_hist, seconds: float) -> dict:
    """Time the CPU restatement of the scipp pipeline on the host cores, on the
    very batch the GPU binned, and check the GPU's histogram against it.

    Main figure: oracle/binning_ref.c (group -> project -> hist -> +=, OpenMP
    over the host cores, the way scipp's TBB kernels run) over the whole step
    batch (1.4e8 events) with this step's replica, repeated until ``seconds``
    of CPU work.  Its first pass is also the parity check of the GPU's current
    histogram for that step (bit-exact).  The single-thread NumPy oracle is
    timed beside it on a 4e6-event slice of the same batch.
    """
    from oracle import c_oracle
    from oracle import scipp_semantics as ora

    # threads: the box's CPU share (OMP_NUM_THREADS, set by the harness), else
    # every core this process may run on
    visible = len(os.sched_getaffinity(0))
    threads = int(os.environ.get('OMP_NUM_THREADS', '0') or 0) or visible
    c = c_oracle.CDetectorView(inst.detector_number, ps, view.n_screen, inst.edges.edges_ns(),
                               threads=threads)
    n = len(pid_h)
    done, t_total, k = 0, 0.0, 0
    bit_exact = None
    while (t_total < seconds and k < 50) or k == 0:
        t0 = time.perf_counter()
        c.accumulate(pid_h, toa_h, replica)
        t_total += time.perf_counter() - t0
        if k == 0:
            ref = c.hist.reshape(gpu_hist.shape)
            bit_exact = bool(np.array_equal(ref.astype(np.float64), gpu_hist))
            ref_total = int(ref.sum())
        done += n
        k += 1
    capped = {'value': done / t_total, 'cores': c.threads_used, 'passes': k, 'seconds': t_total}
    # the same restatement on every CPU this process may run on (the
    # reference's scipp/TBB kernels and job pool use all host cores,
    # core/job_manager.py:304-306); the harness's OMP_NUM_THREADS share above
    every = None
    if visible > c.threads_used:
        ca = c_oracle.CDetectorView(inst.detector_number, ps, view.n_screen, inst.edges.edges_ns(),
                                    threads=visible)
        done_a, t_a, k_a = 0, 0.0, 0
        while (t_a < seconds / 2 and k_a < 50) or k_a == 0:
            t0 = time.perf_counter()
            ca.accumulate(pid_h, toa_h, replica)
            t_a += time.perf_counter() - t0
            done_a += n
            k_a += 1
        every = {'value': done_a / t_a, 'cores': ca.threads_used, 'passes': k_a, 'seconds': t_a}
        del ca
    main = every if every is not None and every['value'] > capped['value'] else capped
    m = min(n, 4_000_000)
    o = ora.OracleDetectorView(
        detector_number=inst.detector_number, pixel_screen=ps,
        screen_shape=tuple(view.screen_shape), toa_edges_ns=inst.edges.edges_ns())
    t0 = time.perf_counter()
    o.batch_histogram(pid_h[:m], toa_h[:m], replica)
    t_np = time.perf_counter() - t0
    return {
        'value': main['value'],
        'unit': 'events/s',
        'cores': main['cores'],
        'cpus_visible': visible,
        'kind': 'port',
        'sample': f'passes over the bench step batch ({n} events, replica {replica}) through '
        f'oracle/binning_ref.c: {capped["passes"]} with {capped["cores"]} OpenMP threads (the harness '
        f'share, OMP_NUM_THREADS) in {capped["seconds"]:.1f} s'
        + (f', {every["passes"]} with {every["cores"]} threads (every visible CPU) in {every["seconds"]:.1f} s'
           if every else '')
        + f'; value = the faster; NumPy oracle (1 core) on {m} events of it: {m / t_np:.3e} events/s',
        'share_threads': capped,
        'all_visible_threads': every,
        'numpy_1core': m / t_np,
        'parity': {'events': n, 'replica': replica, 'bit_exact': bit_exact,
                   'oracle_total': ref_total, 'gpu_total': int(gpu_hist.sum())},
    }


def oracle_pixel_screen(args, inst):
    """The oracle's pixel -> screen index of the bench view (test infrastructure)."""
    from esslivedata_amd import synthetic
    from oracle import scipp_semantics as ora

    if args.view == 'geometric':
        return ora.geometric_pixel_screen(inst.coords, inst.resolution, flip_x=args.workload == 'loki')
    # the oracle's closed-form view index (no transform applied)
    spec = {'mantle_front_layer': ([('module', 'segment', 'counter'), ('strip',)], {'wire': 0}),
            'wire_view': ([('wire',), ('module', 'segment', 'counter')], {}),
            'strip_view': ([('strip',)], {})}[args.view]
    return ora.folded_view_index(synthetic.DREAM_BANK_SIZES['mantle_detector'], *spec)[0][None]


def _profile_entry(workload: str, kernel: str):
    path = ROOT / 'profiles' / f'{PROFILE_ROUND}_{workload}_bench.json'
    try:
        return json.loads(path.read_text())[KERNEL_SYMBOL[kernel]], str(path.relative_to(ROOT))
    except (OSError, KeyError, ValueError):
        return None, None


def profiled_traffic(workload: str, kernel: str):
    """HBM bytes per launch of ``kernel`` from the committed rocprofv3 PMC
    summary of this same bench command (2 x FETCH_SIZE + WRITE_SIZE, the gfx950
    correction of MI355X_MICROARCH.md), or None when no profile is committed."""
    e, src = _profile_entry(workload, kernel)
    if e is None or 'hbm_traffic_bytes' not in e:
        return None
    return {
        'bytes': e['hbm_traffic_bytes'],
        'read': e['hbm_read_bytes'],
        'write': e['hbm_write_bytes'],
        'profiled_avg_ms': e.get('avg_ms_steady', e['avg_ms']),
        'source': src,
        # the committed profile's bench line, from the same traced run
        'traced_line': (src.replace('_bench.json', '_traced_bench_line.json')
                        if (ROOT / src.replace('_bench.json', '_traced_bench_line.json')).exists()
                        else None),
    }


def profiled_lds(workload: str, kernel: str):
    """LDS counters of ``kernel`` per launch from the committed profile, and the
    LDS-atomic efficiency north_star asks for: the fraction of LDS-array cycles
    that are not bank-conflict replays, 1 - SQ_LDS_BANK_CONFLICT /
    SQ_LDS_IDX_ACTIVE (MI355X_MICROARCH.md 'LDS'); conflict cycles per LDS
    instruction beside it."""
    e, src = _profile_entry(workload, kernel)
    pm = (e or {}).get('pmc_per_dispatch', {})
    if 'SQ_INSTS_LDS' not in pm or 'SQ_LDS_BANK_CONFLICT' not in pm:
        return None
    out = {
        'SQ_INSTS_LDS': pm['SQ_INSTS_LDS'],
        'SQ_LDS_BANK_CONFLICT': pm['SQ_LDS_BANK_CONFLICT'],
        'SQ_LDS_IDX_ACTIVE': pm.get('SQ_LDS_IDX_ACTIVE'),
        'conflict_cycles_per_lds_inst': pm['SQ_LDS_BANK_CONFLICT'] / max(pm['SQ_INSTS_LDS'], 1.0),
        'efficiency': None,
        'source': src,
    }
    if pm.get('SQ_LDS_IDX_ACTIVE'):
        out['efficiency'] = 1.0 - pm['SQ_LDS_BANK_CONFLICT'] / pm['SQ_LDS_IDX_ACTIVE']
    return out


def bank_leg(args, rank: int, world: int, dev, stream, steps: int, warmup: int) -> dict | None:
    """Pixel-range (bank) sharding, SURVEY 8(e) axis 2: LOKI's nine banks
    (config/instruments/loki/streams.py:17-27) placed on the ranks with
    ``assign_banks``; each rank bins its banks' event streams with one engine
    per bank (one workflow per bank, as the reference's jobs) and no
    collective touches the data path.  Events per bank and step: pulses x
    events_per_pulse x (bank pixels / bank-0 pixels), uniform over the bank's
    pixels.  Returns the whole-node line fields on rank 0 (None elsewhere),
    with every rank's banks checked bit-exactly against oracle/binning_ref.c."""
    import torch
    import torch.distributed as dist

    from esslivedata_amd import projection, synthetic
    from esslivedata_amd.distributed import assign_banks
    from esslivedata_amd.engine import BinningEngine

    banks = synthetic.LOKI_BANKS
    sizes = {name: hi - lo + 1 for name, (lo, hi) in banks.items()}
    place = assign_banks(sizes, world)
    p0 = sizes['loki_detector_0']
    per_pulse = {name: int(round(args.events_per_pulse * sz / p0)) for name, sz in sizes.items()}
    mine = sorted((name for name, r in place.items() if r == rank), key=lambda n: int(n.rsplit('_', 1)[1]))
    local = []
    for name in mine:
        b = int(name.rsplit('_', 1)[1])
        inst = synthetic.loki_bank(b)
        view = projection.geometric_lut(inst.detector_number, inst.coords, inst.resolution, flip_x=True)
        eng = BinningEngine(toa_edges_ns=inst.edges.edges_ns(), out_lut=view.lut,
                            pid_offset=view.pid_offset, n_screen=view.n_screen,
                            device=dev.index, stream=stream.cuda_stream)
        lo, hi = banks[name]
        n_p = per_pulse[name]
        msgs = []
        for k in range(2):  # two rotated batches per bank
            pid, toa = synthetic.torch_uniform_events(n_p * args.pulses, lo, hi, 500 + 37 * b + k, dev)
            msgs.append((pid, toa, [(pid[p * n_p:(p + 1) * n_p], toa[p * n_p:(p + 1) * n_p])
                                    for p in range(args.pulses)]))
        local.append((name, inst, view, eng, msgs))
    torch.cuda.synchronize(dev)

    def step(i: int) -> None:
        for _, _, view, eng, msgs in local:
            eng.stage_tensors_batch(msgs[i % 2][2])
            eng.accumulate(i % view.n_replicas)
        for *_, eng, _ in local:  # the first waits for the stream, the others find it done
            eng.finalize(images=True)

    for i in range(warmup):
        step(i)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(steps):
        step(warmup + i)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # parity: every rank's banks, one more step each, full current histogram
    # against the C oracle on the same events
    from oracle import c_oracle
    from oracle import scipp_semantics as ora

    threads = int(os.environ.get('OMP_NUM_THREADS', '0') or 0) or len(os.sched_getaffinity(0))
    exact = 1
    for name, inst, view, eng, msgs in local:
        r_chk = (warmup + steps) % view.n_replicas
        eng.stage_tensors_batch(msgs[1][2])
        eng.accumulate(r_chk)
        chk = eng.finalize(hists=True)
        ps = ora.geometric_pixel_screen(inst.coords, inst.resolution, flip_x=True)
        c = c_oracle.CDetectorView(inst.detector_number, ps, view.n_screen, inst.edges.edges_ns(),
                                   threads=threads)
        c.accumulate(msgs[1][0].cpu().numpy(), msgs[1][1].cpu().numpy(), r_chk)
        ref = c.hist.reshape(chk.current_hist.shape).astype(np.float64)
        exact &= int(np.array_equal(ref, chk.current_hist))
        eng.close()
    if world > 1:
        t = torch.tensor([elapsed, -float(exact)], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, exact = float(t[0].item()), int(-t[1].item())
    if rank != 0:
        return None
    total = sum(per_pulse.values()) * args.pulses * steps
    n_step = sum(per_pulse.values()) * args.pulses
    return {
        'value': total / elapsed,
        'unit': 'events/s',
        'ms_per_step': 1e3 * elapsed / steps,
        'steps': steps,
        'events_per_step': n_step,
        'step_frac': (BYTES_PER_EVENT * n_step + 4 * 100 * (20736 + 8 * 3888)) / (elapsed / steps) / 1e9
                     / HBM_PEAK_GBS / world,
        'banks_per_rank': {str(r): sorted(n for n, d in place.items() if d == r) for r in range(world)},
        'placement': 'assign_banks (LPT by pixel count), no collective on the data path',
        'bit_exact_vs_oracle': bool(exact),
        'note': "LOKI's 9 banks (loki/streams.py:17-27), xy_plane views at loki/factories.py:101-112 "
                'resolutions, 5 replicas; events per bank proportional to its pixels '
                f'({args.events_per_pulse} per pulse for bank 0); one engine per bank on each rank',
    }


def bank_main(args, rank: int, world: int, dev) -> None:
    """``--shard banks``: the bank-sharded LOKI leg as the line itself."""
    import torch
    import torch.distributed as dist

    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    leg = bank_leg(args, rank, world, dev, stream, args.steps, args.warmup)
    if rank == 0:
        result = {
            'metric': 'binned events/sec (whole node), DREAM-scale detector view; % HBM roofline',
            'value': leg['value'],
            'unit': 'events/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': leg['ms_per_step'],
            'higher_is_better': True,
            'scaling': 'weak' if world <= 9 else 'strong',
            'vs_baseline': None,
            'dtype': 'int32',
            'data': 'synthetic (seeded ev44-shaped streams generated in HBM; no recorded data offline)',
            'config': {
                'workload': 'loki_9_banks_xy_plane',
                'events_per_step': leg['events_per_step'],
                'pulses_per_step': args.pulses,
                'parallelism': f'bank sharding x{world} (assign_banks, no collective)',
            },
            'bank_sharding': leg,
            'check': {'bit_exact_vs_oracle': leg['bit_exact_vs_oracle']},
        }
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        sys.exit(launch_ranks(args))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get('WORLD_SIZE', '1'))
    if world != args.gpus:
        raise SystemExit(f'bench.py: --gpus {args.gpus} but WORLD_SIZE={world}')
    rank = int(os.environ.get('RANK', '0'))
    # one GPU per rank; more ranks than GPUs (a gloo rehearsal) share them
    local = int(os.environ.get('LOCAL_RANK', '0')) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    if world > 1:
        # RCCL over xGMI; LDE_BENCH_BACKEND=gloo rehearses the multi-rank
        # path with several ranks on one GPU (host-staged collectives)
        backend = os.environ.get('LDE_BENCH_BACKEND', 'nccl')
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)
        else:
            dist.init_process_group(backend)

    from esslivedata_amd import projection, synthetic
    from esslivedata_amd.engine import BinningEngine

    if args.shard == 'banks':
        return bank_main(args, rank, world, dev)
    monitor = args.workload == 'monitor'
    bifrost = args.workload == 'bifrost'
    if (monitor or bifrost) and (args.view != 'geometric' or args.coordinate != 'toa'):
        raise SystemExit(f'--workload {args.workload}: TOA mode, its own view')
    inst = (synthetic.dream_mantle() if args.workload == 'dream' else
            synthetic.loki_bank0() if args.workload == 'loki' else
            synthetic.bifrost_unified() if bifrost else None)
    if inst is not None and (args.num_bins or args.toa_scale or args.toa_start is not None):
        # EdgesModel's reachable TOA configurations (parameter_models.py:82-105)
        inst = synthetic.with_toa_edges(inst, num_bins=args.num_bins, scale=args.toa_scale,
                                        start=args.toa_start)
    from esslivedata_amd.edges import TOAEdges

    if monitor:
        view = None  # the monitor histogram: every event, one TOA axis
    elif bifrost:  # bifrost/specs.py:285-299: (arc, tube) x (channel, pixel), float32
        view = projection.logical_lut(inst.detector_number, transform=synthetic.bifrost_transform)
    elif args.view != 'geometric':
        if args.workload != 'dream' or args.coordinate != 'toa':
            raise SystemExit('--view: DREAM mantle logical views, TOA mode')
        cfg = synthetic.dream_logical_views()[args.view]
        view = projection.logical_lut(inst.detector_number,
                                      transform=lambda a: cfg.transform(a, 'mantle_detector'),
                                      reduction_dim=cfg.reduction_dim)
    else:
        view = projection.geometric_lut(
            inst.detector_number, inst.coords, inst.resolution, flip_x=args.workload == 'loki'
        )
    edges = TOAEdges().edges_ns() if monitor else inst.edges.edges_ns()
    coord = None
    if args.coordinate == 'wavelength':
        from esslivedata_amd import wavelength
        from esslivedata_amd.edges import WavelengthEdges

        tab = synthetic.dream_wavelength_table() if args.workload == 'dream' else \
            wavelength.ideal_lookup_table(27.5, 29.5, 41, 71.5e6, 287)
        src = (0.0, 0.0, -synthetic.DREAM_L1 if args.workload == 'dream' else -23.0)
        lt = wavelength.pixel_ltotal(inst.positions, source_position=src)
        d = wavelength.distance_per_pid(inst.detector_number, lt, view.pid_offset, view.lut.shape[1])
        edges = WavelengthEdges(start=0.2, stop=3.6 if args.workload == 'dream' else 10.0,
                                num_bins=100).get_edges()
        coord = (d, tab, lt)
    # one non-default torch stream for the data generation, the engine and
    # the collectives: everything in order on it, no cross-stream waits
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    if monitor:
        eng = BinningEngine.monitor(edges, device=local, stream=stream.cuda_stream)
    else:
        eng = BinningEngine(
            toa_edges_ns=edges,
            out_lut=view.lut,
            pid_offset=view.pid_offset,
            n_screen=view.n_screen,
            strategy=args.strategy,
            device=local,
            stream=stream.cuda_stream,
            **({'out_dtype': 'float32'} if bifrost else {}),
        )
    n_rep = 1 if monitor else view.n_replicas
    if coord is not None:
        d, tab, _ = coord
        eng.set_coordinate_lut(d, tab.table, dist0=tab.distance0, dist_step=tab.distance_step,
                               time0=tab.time0, time_step=tab.time_step)
    n_pulse = 45 * 1000 if bifrost else args.events_per_pulse  # bifrost/streams.py:22-43
    # BIFROST at the reference cadence: the batch's 14 x 45 bank messages are
    # one push, accumulated once and finalized once per step
    bifrost_batch = bifrost and args.bifrost_cadence == 'batch'
    if bifrost:  # the device symbols of the float32 path (profile lookup)
        KERNEL_SYMBOL['finalize'] = 'k_finalize_f32'
        if bifrost_batch:
            KERNEL_SYMBOL['atomic'] = 'k_bin_atomic_blocks'
    n_step = n_pulse * args.pulses
    n_batches = max(1, args.batches)

    def gen(b: int, r: int = rank):
        """Batch ``b`` of rank ``r`` (seeded; any rank can regenerate another's)."""
        seed = 7 + 1000 * r + 17 * b
        if args.workload == 'dream':
            return synthetic.torch_dream_events(n_step, inst, seed, dev)
        if args.workload == 'loki':
            return synthetic.torch_uniform_events(n_step, 1, 802816, seed, dev)
        g = torch.Generator(device=dev)
        g.manual_seed(seed + 1)
        # fake_monitors.py / fake_detectors.py: TOA normal(30 ms, 10 ms)
        t = (torch.randn(n_step, generator=g, device=dev, dtype=torch.float32) * 10e6 + 30e6).to(
            torch.int32)
        if bifrost:  # uniform ids over the 13,500 pixels
            return synthetic.torch_uniform_events(n_step, 1, 13500, seed, dev)[0], t
        return None, t

    batches = [gen(b) for b in range(n_batches)]
    torch.cuda.synchronize(dev)
    nbins = (1 if monitor else view.n_screen) * eng.n_toa_bins
    bpe_step = MONITOR_BYTES_PER_EVENT if monitor else BYTES_PER_EVENT
    from esslivedata_amd.distributed import OutputReducer, PushReducer

    # N > 1: every rank keeps its own histograms; per finalize only the
    # published outputs (u64 partial images + totals, 2*S + 4 words) are
    # RCCL-reduced onto rank 0 (bit-exact integer sums).  The float32 BIFROST
    # view merges per push instead (PushReducer: the ranks' exact counts of a
    # push summed onto rank 0 before its f32 adds, accumulators.py:129-135)
    reducer = push_reducer = None
    if world > 1:
        if bifrost:
            push_reducer = PushReducer(eng, dev)
        else:
            reducer = OutputReducer(eng, dev)

    # one device buffer view per ev44 message, made once: in the service each
    # message arrives as its own buffer, slicing here is only how the
    # synthetic stream is laid out
    def split(pid, toa):
        return [(None if pid is None else pid[p * n_pulse : (p + 1) * n_pulse],
                 toa[p * n_pulse : (p + 1) * n_pulse]) for p in range(args.pulses)]

    batch_msgs = [split(*bt) for bt in batches]
    if bifrost:  # per pulse one message per bank (300 pixels each), 1,000 events each
        batch_pushes = [[[(pid[p * n_pulse + b * 1000 : p * n_pulse + (b + 1) * 1000],
                           toa[p * n_pulse + b * 1000 : p * n_pulse + (b + 1) * 1000])
                          for b in range(45)] for p in range(args.pulses)] for pid, toa in batches]
        if bifrost_batch:  # one push of all the batch's messages
            batch_pushes = [[[m for push in pushes for m in push]] for pushes in batch_pushes]
        # the messages' device pointers, as they arrive (one descriptor table
        # per push, staged with one call in the step)
        push_tables = [[eng.device_messages(push) for push in pushes] for pushes in batch_pushes]

    # A step bins the batch staged before it, then stages the next batch's
    # messages and finalizes the window: the next pulses' messages reach the
    # staging accumulator while the window's outputs are read back, as in the
    # service, where messages arrive independently of the publish cadence.
    # Every step stages one batch, so the timed region holds K stagings, K
    # accumulates and K finalizes; the batch staged by the last step is binned
    # by the first step after the region.
    # Step i bins batch i % n_batches: consecutive steps never see the same
    # events (a stream's batches differ; per-batch predictions such as PIXEL's
    # slot sizes are exercised as in the service).
    def step(i: int, stage_next: bool = True):
        if bifrost:  # every push is one accumulate (float32 adds in the reference order)
            for table in push_tables[i % n_batches]:
                eng.stage_device_messages(table)
                if push_reducer is not None:
                    push_reducer.push(0)
                else:
                    eng.accumulate(0)
            if rank == 0:
                eng.finalize(images=True)
            return
        eng.accumulate(i % n_rep)
        if stage_next:
            eng.stage_tensors_batch(batch_msgs[(i + 1) % n_batches])
        if reducer is not None:
            reducer.finalize()
        elif args.finalize_overlap:
            # the previous window's outputs are read once this batch's binning
            # is enqueued behind them; this window's finalize is enqueued next
            drain()
            pending[0] = eng.finalize(images=True, wait=False)
        else:
            eng.finalize(images=True)

    pending = [None]

    def drain():  # the outputs of the finalize still pending (every step's are read)
        if pending[0] is not None:
            pending[0].result()
            pending[0] = None

    if not bifrost:
        eng.stage_tensors_batch(batch_msgs[0])
    for i in range(args.warmup):
        step(i)
    drain()
    torch.cuda.synchronize(dev)
    # per-kernel breakdown (every kernel bracketed with HIP events) from 3
    # extra steps before the timed region; the dominant kernel is the one
    # with the largest time per step among them (a kernel, not a strategy:
    # in wavelength mode the coordinate pass dominates the sieve)
    names = ('atomic', 'partition', 'tile_accumulate', 'plan', 'paged', 'page_plan',
             'page_accumulate', 'split', 'split_aux', 'coord', 'pixel', 'monitor', 'binning',
             'finalize', 'wide', 'wide_accumulate')
    eng.timing_select(None)
    eng.timing_enable(True)
    n_prof = 3
    for i in range(n_prof):
        step(args.warmup + i)
    drain()
    torch.cuda.synchronize(dev)
    stats = {k: eng.kernel_stats(k) for k in names}
    info = eng.info()
    eng.timing_enable(False)
    per_step = {k: v[0] / n_prof for k, v in stats.items()
                if v[1] and k in KERNEL_SYMBOL and k != 'binning'}
    dom = max(per_step, key=per_step.get) if per_step else 'split'
    # The timed region stamps only the dominant kernel, by its own dispatch
    # (no marker packets, no extra host calls in front of the launch).  A
    # stamped dispatch still costs step time (hipExtLaunchKernelGGL with
    # events: ~5 us before the next kernel starts plus host time, ~16 us per
    # step on DREAM), so the kernel is stamped on every `timing_stride`-th step
    # of the region, spread over it, and its average is taken over those
    stride = max(1, args.timing_stride)
    untimed = os.environ.get('LDE_BENCH_UNTIMED', '0') not in ('', '0')
    sampled = set() if untimed else set(range(0, args.steps, stride))
    first = args.warmup + n_prof
    eng.timing_select([])
    if world > 1:
        dist.barrier()
    eng.timing_enable(True)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    cpu0 = time.process_time()
    for i in range(args.steps):
        if i in sampled:
            eng.timing_select([dom])
            step(first + i)
            eng.timing_select([])
        else:
            step(first + i)
    drain()  # the last step's outputs, inside the timed region
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    host_cpu_s = time.process_time() - cpu0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    timed = {dom: eng.kernel_stats(dom)}
    eng.timing_enable(False)
    step(first + args.steps, stage_next=False)  # bins the batch the last timed step staged
    drain()
    # the parity legs bin the batch after the last one binned (never a repeat)
    b_chk = (first + args.steps + 1) % n_batches
    pid, toa = batches[b_chk]
    messages = batch_msgs[b_chk]
    pushes = batch_pushes[b_chk] if bifrost else None

    # end-to-end (PCIe-inclusive) leg, reported beside `value`: the same
    # messages as host arrays, staged through lde_stage (copy into the pinned
    # ring + async H2D on the engine stream), binned and finalized
    e2e = None
    if args.e2e_steps > 0 and not (monitor or bifrost):
        from esslivedata_amd.ev44 import serialise_ev44

        t_pulse = 1_767_225_600 * 10**9
        host_msgs = [
            np.frombuffer(serialise_ev44(args.workload, k, [t_pulse + k * 71_428_571], 0,
                                         mt.cpu().numpy(), mp.cpu().numpy()), dtype=np.uint8)
            for k, (mp, mt) in enumerate(messages)
        ]

        def host_step(i: int):
            for payload in host_msgs:
                eng.stage_ev44(payload)
            eng.accumulate(i % view.n_replicas)
            if reducer is not None:
                reducer.finalize()
            else:
                eng.finalize(images=True)

        host_step(0)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        for i in range(args.e2e_steps):
            host_step(1 + i)
        torch.cuda.synchronize(dev)
        e2e_s = time.perf_counter() - t1
        if world > 1:
            t = torch.tensor([e2e_s], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            e2e_s = float(t.item())
        e2e = {
            'value': n_step * args.e2e_steps * world / e2e_s,
            'unit': 'events/s',
            'ms_per_step': 1e3 * e2e_s / args.e2e_steps,
            'steps': args.e2e_steps,
            'note': 'PCIe-inclusive: each step hands its 14 serialized ev44 payloads '
                    '(pageable host bytes) to lde_stage_ev44 (in-place flatbuffer decode, '
                    'memcpy into the pinned ring + async H2D), then accumulate + finalize; '
                    'not `value`',
        }
        del host_msgs
    total_events = n_step * args.steps * world
    value = total_events / elapsed
    ms_per_step = 1e3 * elapsed / args.steps
    step_gbs = (bpe_step * n_step + 4 * nbins) * world / (ms_per_step / 1e3) / 1e9

    # dominant kernel and its roofline (HIP events of the timed region)
    ms, launches = timed[dom]
    # every binning kernel processes all events of the timed steps across its launches
    events_per_launch = n_step * len(sampled) / max(launches, 1)
    alg_bytes = KERNEL_BYTES_PER_EVENT.get(dom, BYTES_PER_EVENT) * events_per_launch
    avg_s = (ms / max(launches, 1)) / 1e3
    achieved = alg_bytes / avg_s / 1e9 if avg_s > 0 else 0.0
    prof_name = ('wavelength' if args.coordinate == 'wavelength' else
                 args.workload if args.view == 'geometric' else args.view)
    if args.num_bins or args.toa_scale or args.toa_start is not None:
        # a non-default TOA binning has its own profile (tools/prof_round.sh NAME=)
        prof_name += f'_t{args.num_bins or "def"}{args.toa_scale or ""}' + (
            f'_s{args.toa_start:g}' if args.toa_start is not None else '')
    traffic = profiled_traffic(prof_name, dom)
    if traffic is not None:
        # per-dispatch tracing slows a kernel: the traced run's own line agrees
        # with its profile; this untraced line records the difference
        traffic['trace_overhead'] = traffic['profiled_avg_ms'] / max(ms / max(launches, 1), 1e-9) - 1.0
    bin_ms, bin_n = stats['binning']  # the extra steps
    n_acc = n_pulse if (bifrost and not bifrost_batch) else n_step  # events one accumulate bins
    pipeline_gbs = bpe_step * n_acc / ((bin_ms / max(bin_n, 1)) / 1e3) / 1e9 if bin_ms else 0.0

    result = {
        'metric': 'binned events/sec (whole node), DREAM-scale detector view; % HBM roofline',
        'value': value,
        'unit': 'events/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': ms_per_step,
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'int32',
        'data': 'synthetic (seeded ev44-shaped streams generated in HBM; no recorded data offline)',
        'config': {
            'workload': ('monitor_toa_histogram' if monitor else 'bifrost_unified_f32' if bifrost else
                         'dream_mantle_cylinder_mantle_z' if args.workload == 'dream'
                         else 'loki_bank0_xy_plane') if args.view == 'geometric'
                        else f'dream_mantle_{args.view}',
            'coordinate': args.coordinate,
            'pixels': 0 if monitor else int(inst.detector_number.size),
            'screen': [1] if monitor else list(view.screen_shape),
            'replicas': n_rep,
            'toa_bins': eng.n_toa_bins,
            'toa_edges': 'linear' if monitor else inst.edges.scale,
            **({} if monitor else {'toa_range_ms': [inst.edges.start, inst.edges.stop]}),
            'events_per_step': n_step,
            'pulses_per_step': args.pulses,
            'strategy': info['last_strategy'],
            **({'bifrost_cadence': args.bifrost_cadence,
                'pushes_per_step': len(batch_pushes[0]),
                'messages_per_push': len(batch_pushes[0][0])} if bifrost else {}),
            'tile_bits': info['tile_bits'],
            # each step's finalize outputs are read after the next batch's
            # binning is enqueued (lde_finalize_begin/_end); every one inside
            # the timed region
            'finalize_overlap': bool(args.finalize_overlap and not bifrost and reducer is None),
            'parallelism': (f'event-batch sharding x{world} + '
                            f'{"RCCL" if dist.get_backend() == "nccl" else dist.get_backend()} '
                            'reduce of partial outputs') if world > 1 else 'single GPU',
        },
        'roofline': {
            'bound': 'hbm',
            'kernel': dom,
            'symbol': KERNEL_SYMBOL.get(dom),  # its device symbol in the rocprofv3 summary
            'achieved': achieved,
            'peak': HBM_PEAK_GBS,
            'unit': 'GB/s',
            'frac': achieved / HBM_PEAK_GBS,
            'traffic': traffic['bytes'] if traffic else None,
            'traffic_detail': traffic,
            'avg_launch_ms': ms / max(launches, 1),
            'launches': launches,
            'timed_steps': len(sampled),
            'launches_note': f'dominant kernel stamped by its own dispatch (HIP events) on '
                             f'{len(sampled)} of the {args.steps} timed steps (every {stride}th); '
                             'the span includes the start marker the runtime enqueues just ahead '
                             'of the kernel (about 10 us), traffic_detail.profiled_avg_ms is the '
                             'rocprofv3 kernel duration',
            'pipeline_achieved': pipeline_gbs,
            'pipeline_frac': pipeline_gbs / HBM_PEAK_GBS,
            # whole step (incl. finalize and host gaps): SURVEY 8(d)'s
            # (8 N + 4 S T) bytes per step (4 N + 4 T for a monitor) over ms_per_step
            'step_achieved': step_gbs,
            'step_frac': step_gbs / HBM_PEAK_GBS,
            'lds': profiled_lds(prof_name, dom),
            'kernel_ms': {k: v[0] / max(v[1], 1) for k, v in stats.items() if v[1]},
            'kernel_ms_note': 'per-kernel breakdown and pipeline_* (the whole binning sequence of '
                              'one accumulate) from 3 extra steps after the timed region',
        },
    }
    # host CPU time (all threads of this process) per timed step: the finalize
    # wait sleeps through most of the GPU work instead of spinning a core
    result['host_cpu_ms_per_step'] = 1e3 * host_cpu_s / args.steps
    if e2e is not None:
        result['end_to_end'] = e2e
    if rank == 0 and world == 1 and monitor:
        # parity leg: one more step's histogram against the NumPy oracle
        # (monitor_workflow.py:90-100 event mode) on the whole batch; the CPU
        # baseline is that oracle timed on a 2e7-event slice (1 core)
        from oracle import scipp_semantics as ora

        eng.stage_tensors_batch(messages)
        eng.accumulate(0)
        chk = eng.finalize(hists=True)
        toa_h = toa.cpu().numpy()
        ref = ora.monitor_histogram(toa_h, edges)
        m = min(len(toa_h), 20_000_000)
        t_c = time.perf_counter()
        ora.monitor_histogram(toa_h[:m], edges)
        t_c = time.perf_counter() - t_c
        result['check'] = {
            'current_total': chk.current_total,
            'bit_exact_vs_oracle': bool(np.array_equal(np.asarray(chk.current_hist).ravel(), ref)),
        }
        if not args.no_cpu_baseline:
            result['cpu_baseline'] = {
                'value': m / t_c, 'unit': 'events/s', 'cores': 1, 'kind': 'port',
                'sample': f'oracle.scipp_semantics.monitor_histogram (NumPy, 1 core) on {m} events '
                          f'of the bench batch, {t_c:.2f} s',
            }
    elif rank == 0 and world == 1 and bifrost:
        # parity leg: one more step (its f32 pushes) from zeroed accumulators
        # against the oracle's float32 per-push sums (accumulators.py:86-163)
        from oracle import scipp_semantics as ora

        eng.clear()
        for push in pushes:
            eng.stage_tensors_batch(push)
            eng.accumulate(0)
        chk = eng.finalize(hists=True)
        pid_h, toa_h = pid.cpu().numpy(), toa.cpu().numpy()
        o = ora.OracleDetectorView(
            detector_number=inst.detector_number,
            pixel_screen=ora.logical_screen_index(inst.detector_number.shape,
                                                  synthetic.bifrost_transform)[0][None],
            screen_shape=(15, 900), toa_edges_ns=edges, dtype=np.float32)
        t_c = time.perf_counter()
        if bifrost_batch:  # one push of the whole batch
            o.accumulate(pid_h, toa_h)
        else:
            for p in range(args.pulses):
                o.accumulate(pid_h[p * n_pulse : (p + 1) * n_pulse], toa_h[p * n_pulse : (p + 1) * n_pulse])
        exp = o.finalize()
        t_c = time.perf_counter() - t_c
        result['check'] = {
            'current_total': float(exp['histogram_current'].sum()),
            'bit_exact_vs_oracle': bool(
                chk.current_hist.dtype == np.float32
                and np.array_equal(chk.current_hist, exp['histogram_current'])
                and np.array_equal(chk.cumulative_hist, exp['histogram_cumulative'])),
        }
        if not args.no_cpu_baseline:
            result['cpu_baseline'] = {
                'value': n_step / t_c, 'unit': 'events/s', 'cores': 1, 'kind': 'port',
                'sample': f'oracle.scipp_semantics.OracleDetectorView (NumPy, 1 core, float32 '
                          f'per-push sums) on one step ({len(pushes)} push(es), {n_step} events), '
                          f'{t_c:.2f} s',
            }
    elif rank == 0 and world == 1 and not args.no_cpu_baseline and coord is None:
        # CPU baseline + parity leg: one more GPU step with the full current
        # histogram read back, then the oracle over the same batch
        from oracle import scipp_semantics as ora

        r_chk = (args.warmup + args.steps + 3) % view.n_replicas
        eng.stage_tensors_batch(messages)
        eng.accumulate(r_chk)
        chk = eng.finalize(hists=True)
        ps = oracle_pixel_screen(args, inst)
        result['cpu_baseline'] = cpu_baseline(inst, ps, view, pid.cpu().numpy(), toa.cpu().numpy(),
                                              r_chk, chk.current_hist, args.cpu_baseline_seconds)
        result['check'] = {
            'current_total': chk.current_total,
            'bit_exact_vs_oracle': result['cpu_baseline']['parity']['bit_exact'],
        }
    elif rank == 0 and world == 1 and coord is not None:
        # wavelength parity leg: a step over the first `check_msgs` messages
        # of the batch, its full current histogram against the NumPy oracle
        # (pixel Ltotal -> bilinear table lookup -> hist on the wavelength
        # edges, oracle.scipp_semantics.wavelength_mode) on the same events
        from oracle import scipp_semantics as ora

        d, tab, lt = coord
        check_msgs = max(1, min(args.pulses, -(-20_000_000 // n_pulse)))
        r_chk = (args.warmup + args.steps + 3) % view.n_replicas
        eng.stage_tensors_batch(messages[:check_msgs])
        eng.accumulate(r_chk)
        chk = eng.finalize(hists=True)
        n_chk = check_msgs * n_pulse
        ps = ora.geometric_pixel_screen(inst.coords, inst.resolution, flip_x=args.workload == 'loki')
        o = ora.OracleDetectorView(
            detector_number=inst.detector_number, pixel_screen=ps,
            screen_shape=tuple(view.screen_shape), toa_edges_ns=edges,
            coordinate=ora.wavelength_mode(lt, tab.table, tab.distance0, tab.distance_step,
                                           tab.time0, tab.time_step))
        t_c = time.perf_counter()
        ref = o.batch_histogram(pid[:n_chk].cpu().numpy(), toa[:n_chk].cpu().numpy(), r_chk)
        t_c = time.perf_counter() - t_c
        result['check'] = {
            'events': n_chk,
            'current_total': chk.current_total,
            'oracle_total': int(ref.sum()),
            'bit_exact_vs_oracle': bool(np.array_equal(ref, chk.current_hist)),
            'oracle': 'oracle.scipp_semantics.wavelength_mode (NumPy, 1 core)',
            'oracle_events_per_s': n_chk / t_c,
        }
        result['cpu_baseline'] = {
            'value': n_chk / t_c, 'unit': 'events/s', 'cores': 1, 'kind': 'port',
            'sample': f'oracle.scipp_semantics wavelength mode (NumPy, 1 core: Ltotal lookup, '
                      f'bilinear table interpolation, hist) on the {n_chk}-event check slice of '
                      f'the bench batch, {t_c:.2f} s',
        }
    elif world > 1 and not (monitor or bifrost) and coord is None:
        # parity leg of the sharded path: every rank bins batch b_chk of its own
        # stream, the reducer merges the ranks' outputs onto the root (RCCL),
        # and the root checks the merged current image and totals against
        # oracle/binning_ref.c run over every rank's batch
        r_chk = (args.warmup + args.steps + 3) % view.n_replicas
        eng.stage_tensors_batch(messages)
        eng.accumulate(r_chk)
        merged = reducer.finalize()
        if rank == 0:
            from oracle import c_oracle

            threads = int(os.environ.get('OMP_NUM_THREADS', '0') or 0) or len(os.sched_getaffinity(0))
            c = c_oracle.CDetectorView(inst.detector_number, oracle_pixel_screen(args, inst),
                                       view.n_screen, inst.edges.edges_ns(), threads=threads)
            for r in range(world):  # regenerate rank r's batch b_chk on this device
                p_r, t_r = gen(b_chk, r)
                c.accumulate(p_r.cpu().numpy(), t_r.cpu().numpy(), r_chk)
                del p_r, t_r
            ref = c.hist.reshape(view.n_screen, eng.n_toa_bins)
            cur, _, totals = merged
            result['check'] = {
                'events': n_step * world,
                'ranks': world,
                'current_total': totals[0],
                'oracle_total': int(ref.sum()),
                'bit_exact_vs_oracle': bool(np.array_equal(ref.sum(axis=1).astype(np.float64), cur)
                                            and totals[0] == int(ref.sum())),
                'compared': 'merged current image and current total (RCCL reduce of every '
                            "rank's partial outputs) vs oracle/binning_ref.c over all ranks' batches",
            }
        dist.barrier()
    if (args.bank_steps > 0 and args.workload == 'dream' and args.view == 'geometric'
            and coord is None):
        # the second 8(e) axis beside the event-batch-sharded line: LOKI's banks
        # placed on the ranks, no collective (every rank takes part)
        eng.close()
        del batches, batch_msgs
        torch.cuda.empty_cache()
        leg = bank_leg(args, rank, world, dev, stream, args.bank_steps, 2)
        if rank == 0:
            result['bank_sharding'] = leg
    if rank == 0:
        print(json.dumps(result), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
