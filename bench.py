#!/usr/bin/env python3
"""Benchmark: validated candidates/s of the MI355X validator on the force-free depth-4 batch,
and the wall time to recover the 7 force-free paper solutions at depth 4.

Workload (BASELINE.json configs[2], "force_free --max-depth 4 on 1xMI355X"):
the 142,004 candidates of the reference's depth-4 force-free stream that pass its pre-validate
filters (tests/golden/streams/force_free_d4_validated.txt.gz, compiled once into
data/force_free_d4_validated.npz), tiled and shuffled with seed 0 into --n candidates per GPU.
One "step" = one validation pass of the whole batch: every candidate's program is evaluated
in jets at the reference point and on the 64x64 (rho, z) grid (4097 points), the foliation
determinant and its scaled zero test are applied and the verdict bitmap + per-candidate
outputs are written to HBM.  Inputs are resident in HBM before timing starts.

Multi-GPU (torchrun, one process per GPU): the global batch (--n per rank) is cut into
contiguous shards balanced by the programs' FLOP model (pdeval.shard); every rank validates its
own shard (weak scaling, no data-path collective); after timing, one RCCL all-gather of the
verdict bitmaps (pdeval_gather_bits, through the C ABI) assembles the global result on every
rank, checked against torch.distributed's all-gather.
"""
import argparse
import glob
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'pde-engine_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))

FP64_PEAK_TFLOPS = 78.6      # MI355X FP64 vector peak (spec; MI355X_MICROARCH.md lists FP32 157.3 = 2x)
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md "HBM3E peak BW 8.0 TB/s"
# pass 1 (force-free, full-batch instance, Omega = 0); Kerr: grid_kernel<1, false, false>
DOMINANT = 'grid_kernel<0, false, false>'


_T0 = time.perf_counter()


def log(msg):
    """A progress line on stderr (the JSON result is the only stdout line): every leg reports,
    so no stretch of the run is silent for minutes."""
    print(f'[bench {time.perf_counter() - _T0:7.1f}s] {msg}', file=sys.stderr, flush=True)


# host-measured stages before validation (recorded, not re-run by the bench): the reference's
# enumeration + normalization of the depth-4 force-free stream on one core (SURVEY.md section 6 /
# 8d, stream_generate), and the pre-validate filters over that whole stream on the SymPy pool
ENUM_D4_S = 675.0
PREFILTER_RECORD = os.path.join('profiles', 'r05_prefilter_d4.json')


def time_to_7_end_to_end(validation_s):
    """time_to_7_end_to_end_s: the recorded host stages plus this run's
    validation time, labelled host-measured -- the SymPy work the north star keeps on the host."""
    try:
        with open(os.path.join(ROOT, PREFILTER_RECORD)) as f:
            pf = json.load(f)
    except OSError:
        return {'time_to_7_end_to_end_s': None}
    total = ENUM_D4_S + pf['wall_s'] + validation_s
    return {'time_to_7_end_to_end_s': round(total, 1),
            'time_to_7_end_to_end_parts': {
                'enumeration_normalize_s': ENUM_D4_S, 'enumeration_source': 'SURVEY.md section 6 (reference, 1 core)',
                'prefilters_s': pf['wall_s'], 'prefilters_source': f"{PREFILTER_RECORD} ({pf['procs']} SymPy processes, "
                                                                  f"{pf['rows']} rows, kept == reference: {pf['kept_equals_reference']})",
                'validation_s': round(validation_s, 4), 'validation_source': 'this run',
                'label': 'host-measured recorded stages + measured validation'}}


class heartbeat:
    """A progress line every ``every`` seconds while a long leg runs (a leg whose work is in
    SymPy pool processes or a C call prints nothing of its own for minutes)."""

    def __init__(self, what, every=30.0):
        import threading
        self.what, self.every, self.stop = what, every, threading.Event()
        self.t = threading.Thread(target=self._beat, daemon=True)

    def _beat(self):
        t0 = time.perf_counter()
        while not self.stop.wait(self.every):
            log(f'... {self.what}: {time.perf_counter() - t0:.0f} s')

    def __enter__(self):
        log(self.what)
        self.t.start()
        return self

    def __exit__(self, *exc):
        self.stop.set()
        self.t.join(5)
        return False


def load_workload(problem):
    # force-free: the depth-4 validated set; Kerr: the whole depth<=4 stream
    # (1,024,799 candidates; the pre-validate filters keep 1,999 of a 2,000 seeded sample, so
    # the stream is what reaches validate to 0.05 %: tests/golden/streams/)
    from pdeval.workload import load_programs
    for name in (f'{problem}_d4_validated.npz', f'{problem}_d4_stream.npz',
                 f'{problem}_d3_validated.npz'):
        if os.path.exists(os.path.join(ROOT, 'data', name)):
            return (name,) + tuple(load_programs(name))
    raise FileNotFoundError(f'data/{problem}_d*_*.npz missing')


def _pmc_pass1(k, n_cand, n_batch):
    """Pass-1 candidates of the profiled launch: recorded by scripts/pmc_summary.py from the
    profiled run's own bench line, or (older summaries) its launched waves scaled by this
    batch's pass-1 share -- the same workload, tiled and shuffled the same way."""
    return k.get('pass1_candidates') or k['candidates'] * (n_cand / max(1, n_batch))


def pmc_traffic(n_per_launch, dominant=DOMINANT, n_batch=None):
    """HBM bytes per launch of the dominant kernel from the newest committed PMC summary
    (profiles/*_pmc.json, written by scripts/pmc_summary.py from separate rocprofv3 --pmc
    passes), per pass-1 candidate of the profiled launch, scaled to this launch's pass-1
    candidates; None if there is none."""
    files = sorted(glob.glob(os.path.join(ROOT, 'profiles', '*_pmc.json')))
    for path in reversed(files):          # the newest summary (by name) that has the kernel
        with open(path) as f:
            s = json.load(f)
        kern = s.get('kernels', {})
        # summaries from before the ROT instances name the kernel without its third argument
        k = kern.get(dominant) or kern.get(dominant.replace(', false, false>', ', false>'))
        if k and k.get('candidates') and 'hbm_bytes_per_launch' in k:
            per = k['hbm_bytes_per_launch'] / _pmc_pass1(k, n_per_launch, n_batch or n_per_launch)
            return per * n_per_launch, os.path.basename(path)
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--n', type=int, default=1 << 21,
                    help='candidates per GPU per step (8 GPUs: 2^24, the C4 batch of SURVEY.md §8d)')
    ap.add_argument('--problem', default='force_free')
    ap.add_argument('--early-exit', action='store_true',
                    help='headline run stops after the point stage for point-rejects')
    ap.add_argument('--cpu-seconds', type=float, default=12.0, help='CPU-baseline time budget')
    ap.add_argument('--no-cpu', action='store_true')
    ap.add_argument('--sympy-seconds', type=float, default=120.0,
                    help='wall budget of the SymPy CPU leg (the north star\'s CPU baseline)')
    ap.add_argument('--cpu-procs', type=int, default=0,
                    help='host processes of the SymPy leg (0: OMP_NUM_THREADS, the box\'s CPU share)')
    ap.add_argument('--no-extras', action='store_true',
                    help='skip the early-exit / host-buffer / time-to-solutions legs')
    ap.add_argument('--strict-full', action='store_true',
                    help="only the streaming 'strict' symbolic mode over every validated d4 string "
                         "through the worker pipeline (a steady-state rate; minutes), as one JSON line")
    ap.add_argument('--part', type=int, default=0, help='--strict-full: this share of the set')
    ap.add_argument('--parts', type=int, default=1, help='--strict-full: shares of the set')
    ap.add_argument('--plan-only', action='store_true',
                    help='print every rank\'s environment and shard plan as JSON and exit before any GPU call')
    a = ap.parse_args()
    if a.gpus < 1:
        ap.error('--gpus must be >= 1')
    env_world = os.environ.get('WORLD_SIZE')
    if env_world is None and a.gpus > 1:
        # no launcher around us: start one rank process per GPU ourselves, before this process
        # touches the GPU (the reference's counterpart: N validator processes on one queue,
        # general_method_paper_reproduction.py:802-823)
        sys.exit(launch_ranks(a.gpus, sys.argv[1:]))
    if env_world is not None and int(env_world) != a.gpus:
        print(f'bench.py: --gpus {a.gpus} but WORLD_SIZE={env_world}', file=sys.stderr)
        sys.exit(2)
    if a.plan_only:
        print(json.dumps(plan_record(a)))
        return
    if a.strict_full:
        from pdeval import hostpool
        hostpool.start()
        print(json.dumps(strict_full(part=a.part, parts=a.parts)))
        return
    if not a.no_extras and int(os.environ.get('WORLD_SIZE', '1')) == 1 and a.problem == 'force_free':
        # the worker leg's SymPy pool for the strings the native compiler declines: forked now,
        # before this process touches the GPU (pdeval/hostpool.py)
        from pdeval import hostpool
        hostpool.start()

    import torch
    import torch.distributed as dist
    from pdeval import _lib
    from pdeval.opcodes import PROBLEM_FORCE_FREE, PROBLEM_KERR
    from pdeval.shard import gather_verdicts, gather_verdicts_native, init_native_comm, pack_bits

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        dist.init_process_group('nccl', device_id=torch.device(f'cuda:{local}'))
    torch.cuda.set_device(local)
    dev = torch.device(f'cuda:{local}')
    pid = PROBLEM_FORCE_FREE if a.problem == 'force_free' else PROBLEM_KERR

    log(f'loading {a.problem} workload, {a.n} candidates per GPU')
    pb = ProblemBench(pid, a.n, world, rank, local, dev)
    log('workload resident in HBM')
    slug, ctx, idx, n, ranges = pb.slug, pb.ctx, pb.idx, pb.n, pb.ranges
    ops, off, ops_all, off_all, exprs_all, nprog = pb.ops, pb.off, pb.ops_all, pb.off_all, pb.exprs_all, pb.nprog
    total = a.n * world
    prm = _lib.default_params(pid)
    prm.full_grid = 0 if a.early_exit else 1

    elapsed, kern_ms = pb.timed(prm, a.steps, a.warmup)
    log(f'timed: {a.steps} steps, {elapsed / a.steps * 1e3:.2f} ms per step')

    # After the timed region: the final (plugin) verdicts of this rank's shard -- the device
    # outputs through the host steps (pdeval.shard.final_verdicts, once per distinct program of
    # the tiled batch) -- then the one exchange step, an all-gather of the re-packed bitmaps over
    # RCCL through the C ABI (pdeval_gather_bits), checked against torch.distributed's.
    dev_out = pb.host_outputs()
    status_dev = dev_out['status'].copy()
    if world > 1 or not a.no_extras:
        t0 = time.perf_counter()
        final = pb.final_verdicts(dev_out, prm)
        t_host = time.perf_counter() - t0
        log(f'final verdicts (host steps) {t_host:.2f} s')
        gather = {'bits': 'final (device + host steps)', 'host_steps_s': round(t_host, 3),
                  'host_step_changes_local': int((dev_out['status'] != status_dev).sum())}
    else:   # (--no-extras at one GPU: timing runs, the device bitmap as it stands)
        final = status_dev == 0
        gather = {'bits': 'device (--no-extras)'}
    if world > 1:
        bits = torch.from_numpy(pack_bits(final)).to(dev)
        verdict_all = gather_verdicts(bits, ranges)
        try:
            init_native_comm(ctx, rank, world)
            t0 = time.perf_counter()
            native = gather_verdicts_native(ctx, bits, ranges)
            gather.update(native_rccl_ms=round((time.perf_counter() - t0) * 1e3, 3),
                          native_equals_torch=bool(np.array_equal(native, verdict_all)))
            verdict_all = native
        except Exception as e:   # noqa: BLE001 -- reported; the torch gather result stands
            gather['native_rccl_error'] = str(e)[:200]
    else:
        verdict_all = final
    status = dev_out['status']
    if not a.no_extras and rank == 0:
        # the single-process plugin's verdicts on the same global batch: every distinct program
        # once through pdeval_validate_batch + the host steps, mapped onto the tiled batch
        plugin = pb.plugin_verdicts(prm)[pb.tiled]
        log('plugin verdicts')
        gather['final_equals_plugin'] = bool(np.array_equal(verdict_all, plugin))
        gather['device_bits_equal_plugin'] = None if world > 1 else bool(
            np.array_equal(np.unpackbits(pb.outs['verdict_bits'].cpu().numpy(), bitorder='little')[:n].astype(bool),
                           plugin))

    # size-independent checks at full size: duplicates of one program (the batch is tiled)
    # get one class, and the streamable paper solutions are accepted wherever they occur
    first = np.full(nprog, 255, dtype=np.int16)
    first[idx[::-1]] = status_dev[::-1]
    consistent = bool(np.array_equal(first[idx], status_dev))

    prof = pb.profile(prm, a.steps)
    log('per-pass profile')

    res = None
    if rank == 0:
        value = total * a.steps / elapsed
        res = {
            'metric': ('validated candidates/sec (force-free depth-4 batch, 64x64 grid + p*)'
                       if pid == PROBLEM_FORCE_FREE else
                       'validated candidates/sec (Kerr depth<=4 batch, 64x64 grid + 3 reference points)'),
            'value': value, 'unit': 'candidates/s', 'n_gpus': world, 'steps': a.steps,
            'warmup': a.warmup, 'ms_per_step': elapsed / a.steps * 1e3, 'higher_is_better': True,
            'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f64', 'data': 'synthetic',
            'config': {'workload': f'{slug} validated candidates ({pb.wname}, {nprog} '
                                   f'programs) tiled+shuffled(seed 0) to {a.n}/GPU; 64x64 grid + ref point',
                       'problem': a.problem, 'candidates_per_gpu': a.n, 'points_per_candidate': pb.npts,
                       'full_grid': not a.early_exit, 'parallelism': f'shard{world}'},
            'roofline': prof['roofline'],
            'roofline_hbm': pb.roofline_hbm(kern_ms),
            'pass_ms': prof['pass_ms'],
            'work_lists': prof['counts'],
            'accepted': int(verdict_all.sum()),
            'accepted_device_bits': int((status_dev == 0).sum()) if world == 1 else None,
            'status_hist': np.bincount(status, minlength=8).tolist(),
            'duplicates_consistent': consistent,
            'gather': gather,
        }
        if world > 1:
            res['shard_balance'] = 'flops'
        if not a.no_extras and world == 1 and pid == PROBLEM_FORCE_FREE:
            # configs[4]'s operator on the same build, measured by the driver's own command:
            # the Kerr depth<=4 stream at the same per-GPU batch (the weakest kernel, pass 1)
            with heartbeat('Kerr sub-record'):
                res['kerr'] = kerr_subrecord(a.n, a.steps, a.warmup, world, rank, local, dev)
            log('Kerr sub-record done')

    if not a.no_extras and world == 1:
        log('early-exit / host-buffer / time-to-solutions legs')
        # the reference's control flow: stop after the point stage for point-rejects (same
        # verdicts; reported beside, never as, the headline value)
        pe = _lib.default_params(pid)
        pe.full_grid = 0
        bits_full = pb.outs['verdict_bits'].clone()
        el_e, _ = pb.timed(pe, a.steps, 1)
        same = bool(torch.equal(bits_full, pb.outs['verdict_bits']))
        res['value_early_exit'] = total * a.steps / el_e
        res['early_exit_verdicts_identical'] = same
        # host buffers in and out (PCIe-inclusive), one synchronous C-ABI call
        t0 = time.perf_counter()
        ctx.validate(ops, off, prm)
        res['value_host_buffers'] = n / (time.perf_counter() - t0)
        # wall time to the 7 force-free paper solutions at depth 4 (BASELINE.json metric)
        if pid == PROBLEM_FORCE_FREE:
            from pdeval import problem_defs as P
            from pdeval.discovery import find_known_solutions
            t0 = time.perf_counter()
            rec = find_known_solutions(ctx, P.force_free(), ops_all, off_all, exprs_all)
            res['time_to_7_solutions_s'] = time.perf_counter() - t0
            res['solutions_found'] = rec.n_found
            res['solutions'] = {k: v for k, v in rec.found.items()}
            res['solution_stream_hits'] = rec.stream_hits
            res['time_to_7_breakdown_s'] = {k: round(v, 4) for k, v in rec.seconds.items()}
            res.update(time_to_7_end_to_end(res['time_to_7_solutions_s']))
            # the same, starting from the candidate strings instead of compiled programs: the
            # native compiler (csrc/pdcompile.cpp) plus SymPy for the strings it declines
            from pdeval import native
            strs = [str(s) for s in exprs_all]
            t0 = time.perf_counter()
            _, _, st_n = native.compile_native(pid, strs)
            t_nat = time.perf_counter() - t0
            t0 = time.perf_counter()
            cst = {}
            s_ops, s_off, _ = native.compile_strings(P.force_free(), strs, stats=cst)
            t_comp = time.perf_counter() - t0
            rec2 = find_known_solutions(ctx, P.force_free(), s_ops, s_off, exprs_all)
            res['time_to_7_from_strings_s'] = time.perf_counter() - t0
            res['solutions_found_from_strings'] = rec2.n_found
            res['compile_from_strings'] = {
                'strings': len(strs), 'native': cst['native'], 'sympy_fallback': cst['host'],
                'native_only_s': round(t_nat, 4), 'native_strings_per_s': round(len(strs) / t_nat),
                'hybrid_compile_s': round(t_comp, 4)}

    if not a.no_extras and world == 1 and pid == PROBLEM_FORCE_FREE:
        with heartbeat('strict-mode leg'):
            res['strict'] = strict_leg(exprs_all, local)
        res['value_strict'] = res['strict']['value_strict']
        # the worker pool's batch path, queue tuples in -> result tuples out (the reference's
        # _parallel_validator_worker protocol, general_method_paper_reproduction.py:1756-1816)
        with heartbeat('worker / inline legs'):
            res['worker_process_batch'] = worker_throughput(exprs_all)

    if rank == 0:
        if not a.no_cpu and world == 1:
            procs = a.cpu_procs or int(os.environ.get('OMP_NUM_THREADS', '0') or os.cpu_count())
            if pid == PROBLEM_FORCE_FREE:
                with heartbeat(f'SymPy CPU baseline ({a.sympy_seconds:.0f} s budget, {procs} processes)'):
                    res['cpu_baseline'] = cpu_baseline_sympy(procs, a.sympy_seconds)
            log('C-oracle CPU baseline')
            res['cpu_baseline_c_port'] = cpu_baseline(pid, ops_all, off_all, idx, a.cpu_seconds)
        print(json.dumps(res))
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


class ProblemBench:
    """One problem's workload on this rank's GPU: the tiled batch's shard resident in HBM, the
    library context, the output buffers and the launch stream the events are recorded on."""

    def __init__(self, pid, n_per_rank, world, rank, local, dev):
        import torch
        from pdeval import _lib
        from pdeval.opcodes import PROBLEM_FORCE_FREE, FP_N
        from pdeval import workload as WL
        self.pid, self.world, self.rank, self.dev = pid, world, rank, dev
        self.slug = 'force_free' if pid == PROBLEM_FORCE_FREE else 'kerr_magnetosphere'
        self.dominant = f'grid_kernel<{pid}, false, false>'
        self.wname, self.ops_all, self.off_all, self.exprs_all = load_workload(self.slug)
        self.nprog = len(self.off_all) - 1
        # (experiment PD_BENCH_STREAM_ORDER: keep the stream order)
        self.tiled = WL.tiled_indices(self.nprog, n_per_rank * world, seed=0,
                                      shuffle=not os.environ.get('PD_BENCH_STREAM_ORDER'))
        # algorithmic work of the batch; it also balances the shards
        self.flops_prog = WL.flops_per_program(pid, self.ops_all, self.off_all)
        # the part the lean passes evaluate once per grid row (hoisted x-only prefixes, DESIGN.md
        # §3), unless the library runs with PDEVAL_HOIST=0
        self.hoist = os.environ.get('PDEVAL_HOIST', '1') != '0'
        self.flops_hoist = WL.flops_per_program(pid, self.ops_all, self.off_all, hoisted=True) \
            if self.hoist else np.zeros_like(self.flops_prog)
        plan = WL.rank_plan(self.tiled, world, rank, self.flops_prog)
        self.ranges, self.idx, self.n = plan.ranges, plan.idx, plan.n
        self.ops, self.off = WL.gather_programs(self.ops_all, self.off_all, self.idx)
        self.ctx = _lib.Context(pid, device=local)
        self.npts, self.nref = self.ctx.n_points, self.ctx.n_ref
        out_bytes_per = 1 + 8 + 8 * self.nref + 8 + 4 + 4 + 8 * FP_N + 1.0 / 8
        self.bytes_step = self.ops.nbytes + self.off.nbytes + self.n * out_bytes_per
        n = self.n
        self.d_ops = torch.from_numpy(self.ops).to(dev)
        self.d_off = torch.from_numpy(self.off).to(dev)
        self.outs = dict(verdict_bits=torch.zeros(((n + 31) // 32) * 4, dtype=torch.uint8, device=dev),
                         status=torch.zeros(n, dtype=torch.uint8, device=dev),
                         q_ref=torch.zeros(n, dtype=torch.float64, device=dev),
                         res_ref=torch.zeros(n * self.nref, dtype=torch.float64, device=dev),
                         q_grid=torch.zeros(n, dtype=torch.float64, device=dev),
                         n_bad=torch.zeros(n, dtype=torch.int32, device=dev),
                         n_nonfinite=torch.zeros(n, dtype=torch.int32, device=dev),
                         fingerprint=torch.zeros(n * FP_N, dtype=torch.float64, device=dev))
        self.d_out = _lib.Outputs(*[self.outs[f].data_ptr() for f, _ in _lib.Outputs._fields_])
        # all uploads / zero-fills above ran on torch's default stream: finish them, then run the
        # hot path on a dedicated stream that the events below are recorded on
        torch.cuda.synchronize(dev)
        self.stream = torch.cuda.Stream(dev)

    def step(self, p):
        self.ctx.validate_device(self.d_ops.data_ptr(), self.d_ops.numel(), self.d_off.data_ptr(), self.n,
                                 self.d_out, params=p, stream=self.stream.cuda_stream, zero_bits=True)

    def timed(self, p, steps, warmup):
        """(max over ranks of the wall time of `steps` steps, mean event time of one step)"""
        import torch
        import torch.distributed as dist
        dev = self.dev
        for _ in range(warmup):
            self.step(p)
        torch.cuda.synchronize(dev)
        if self.world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(steps)]
        t0 = time.perf_counter()
        for s, e in ev:
            s.record(self.stream)
            self.step(p)
            e.record(self.stream)
        torch.cuda.synchronize(dev)
        if self.world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        # the last step's device error word (pdeval_device_error: a work-list entry outside the
        # batch would have been skipped silently): raises if it is set
        self.ctx.device_error()
        kern = float(np.mean([s.elapsed_time(e) for s, e in ev]))
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        if self.world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item()), kern

    def host_outputs(self) -> dict:
        """The device outputs of the last step as host arrays (res_ref, fingerprint 2-D)."""
        r = {k: v.cpu().numpy() for k, v in self.outs.items() if k != 'verdict_bits'}
        r['res_ref'] = r['res_ref'].reshape(self.n, self.nref)
        r['fingerprint'] = r['fingerprint'].reshape(self.n, -1)
        r['verdict'] = r['status'] == 0
        return r

    def _kerr(self):
        from pdeval.opcodes import PROBLEM_KERR
        from pdeval._lib import default_kerr_constants
        return default_kerr_constants() if self.pid == PROBLEM_KERR else None

    def final_verdicts(self, r, prm):
        """This rank's final verdicts: its device outputs through the host steps, once per
        distinct program of the shard (pdeval.shard.final_verdicts)."""
        from pdeval import problem_defs as P
        from pdeval.shard import final_verdicts
        items = _LazyItems(self.exprs_all, self.idx)
        return final_verdicts(P.get(self.slug), self._kerr(), prm, self.npts - self.nref, items, r,
                              self.ops, self.off, keys=self.idx)

    def plugin_verdicts(self, prm) -> np.ndarray:
        """The single-process plugin's verdict of every program of the table: one
        pdeval_validate_batch from host buffers + the host steps (BatchValidator's path)."""
        from pdeval import problem_defs as P
        from pdeval.batch import apply_host_steps
        r = self.ctx.validate(self.ops_all, self.off_all, prm)
        apply_host_steps(P.get(self.slug), self._kerr(), prm, self.npts - self.nref,
                         _LazyItems(self.exprs_all, None), r, self.ops_all, self.off_all)
        return np.asarray(r['verdict'], dtype=bool)

    def profile(self, prm, steps) -> dict:
        """Per-pass device times (library HIP events on the launch stream) and the dominant
        kernel's roofline: pass 1 = programs of stack <= 2 in real arithmetic."""
        from pdeval.opcodes import PROBLEM_FORCE_FREE, FLAG_COMPLEX
        ctx = self.ctx
        ctx.set_timing(True)
        pass_ms = {}
        for _ in range(steps):
            self.step(prm)
            for k, v in ctx.pass_times().items():
                pass_ms[k] = pass_ms.get(k, 0.0) + v / steps
        counts = ctx.pass_counts()
        ctx.set_timing(False)
        hdr = self.ops[self.off[:-1]].astype(np.int64)
        depth = (hdr >> 8) & 0xff
        cflag = (hdr & FLAG_COMPLEX) != 0
        in_p1 = (depth <= 2) & ~cflag
        # per candidate: its program's flops at every point, less the hoisted prefix, which runs
        # once per grid row (64 rows of the default grid)
        rows = 64
        fh = self.flops_hoist[self.idx]
        fl = (self.flops_prog[self.idx] - fh) * self.npts + fh * rows
        # candidates pass 1 re-routed to the complex pass after the point stage: their grid work
        # is not pass 1's (charged at the pass-1 mean, a conservative correction)
        rerouted = max(0, counts['complex'] - int(cflag.sum())) if self.pid == PROBLEM_FORCE_FREE else 0
        p1_flops = float(fl[in_p1].sum()) - rerouted * float(fl[in_p1].mean() if in_p1.any() else 0.0)
        p1_ms = pass_ms['pass1_stack2']
        achieved_tf = p1_flops / (p1_ms * 1e-3) / 1e12
        n_p1 = int(in_p1.sum()) - rerouted
        traffic, traffic_src = pmc_traffic(n_p1, self.dominant, self.n)
        roof = {'bound': 'valu_fp64', 'kernel': self.dominant, 'achieved': achieved_tf,
                'peak': FP64_PEAK_TFLOPS, 'unit': 'TFLOP/s', 'frac': achieved_tf / FP64_PEAK_TFLOPS,
                'traffic': traffic, 'traffic_source': traffic_src,
                'kernel_ms': p1_ms, 'kernel_candidates': n_p1,
                'flops_per_launch': p1_flops,
                'flops_model': 'hoisted prefixes once per row' if self.hoist else 'every opcode at every point'}
        roof['traffic_per_candidate'] = traffic / n_p1 if traffic else None
        roof.update(pmc_flop_frac(self.dominant, n_p1, p1_ms, self.n))
        if roof.get('counter_flops_per_candidate'):
            # the FLOP model against the executed FP64 operations
            roof['model_flops_per_candidate'] = p1_flops / max(1, n_p1)
            roof['model_over_counters'] = roof['model_flops_per_candidate'] / roof['counter_flops_per_candidate']
        return {'roofline': roof, 'pass_ms': {k: round(v, 3) for k, v in pass_ms.items()}, 'counts': counts}

    def roofline_hbm(self, kern_ms) -> dict:
        achieved_gbs = self.bytes_step / (kern_ms * 1e-3) / 1e9
        return {'bound': 'hbm', 'achieved': achieved_gbs, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                'frac': achieved_gbs / HBM_PEAK_GBS, 'bytes_per_step': self.bytes_step, 'step_ms': kern_ms}

    def close(self):
        self.ctx.close()


class _LazyItems:
    """exprs[idx[i]] as a read-only sequence of str (the tiled batch's candidate strings,
    without a 2^21-element list)."""

    def __init__(self, exprs, idx):
        self.exprs, self.idx = exprs, idx

    def __len__(self):
        return len(self.exprs) if self.idx is None else len(self.idx)

    def __getitem__(self, i):
        return str(self.exprs[i if self.idx is None else self.idx[i]])


def kerr_subrecord(n, steps, warmup, world, rank, local, dev):
    """configs[4]'s operator (Kerr depth <= 4 stream, 2^21 candidates per GPU) on the same build,
    in the default bench run: value, per-pass times and the pass-1 roofline."""
    from pdeval import _lib
    from pdeval.opcodes import PROBLEM_KERR
    kb = ProblemBench(PROBLEM_KERR, n, world, rank, local, dev)
    try:
        prm = _lib.default_params(PROBLEM_KERR)
        el, kern_ms = kb.timed(prm, steps, warmup)
        prof = kb.profile(prm, steps)
        return {'metric': 'validated candidates/sec (Kerr depth<=4 batch, 64x64 grid + 3 reference points)',
                'value': kb.n * world * steps / el, 'unit': 'candidates/s', 'ms_per_step': el / steps * 1e3,
                'workload': f'{kb.wname} ({kb.nprog} programs) tiled+shuffled(seed 0) to {n}/GPU',
                'roofline': prof['roofline'], 'pass_ms': prof['pass_ms'], 'work_lists': prof['counts']}
    finally:
        kb.close()


def pmc_flop_frac(dominant, n_cand, kernel_ms, n_batch):
    """The dominant kernel's FP64 FLOP rate from the hardware counters (the newest committed
    PMC summary with SQ FP64 counts: (2 FMA + MUL + ADD) x 64 lanes, per launch, divided by the
    pass-1 candidates of the profiled launch -- not by its launched waves, which include the
    candidates pass 1 hands on -- then scaled to this launch's pass-1 candidates and its event
    time), beside the FLOP model's fraction; {} when no summary has them.  (TRANS -- rcp, sqrt
    estimates -- is not counted as FLOPs.)"""
    files = sorted(glob.glob(os.path.join(ROOT, 'profiles', '*_pmc.json')))
    for path in reversed(files):
        with open(path) as f:
            s = json.load(f)
        k = s.get('kernels', {}).get(dominant) or s.get('kernels', {}).get(dominant.replace(', false, false>', ', false>'))
        if k and k.get('candidates') and 'SQ_INSTS_VALU_FMA_F64' in k:
            fl = 64.0 * (2 * k['SQ_INSTS_VALU_FMA_F64'] + k.get('SQ_INSTS_VALU_MUL_F64', 0.0) +
                         k.get('SQ_INSTS_VALU_ADD_F64', 0.0))
            per = fl / _pmc_pass1(k, n_cand, n_batch)
            tf = per * n_cand / (kernel_ms * 1e-3) / 1e12
            return {'counter_flops_per_candidate': per, 'counter_achieved': tf,
                    'counter_frac': tf / FP64_PEAK_TFLOPS, 'counter_source': os.path.basename(path)}
    return {}


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def launch_ranks(n, argv):
    """Run this script as `n` rank processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set as
    torchrun sets them, rendezvous on 127.0.0.1) and return the first non-zero exit status.  The
    parent never imports torch: the ranks are children started before any GPU call here.  If a
    rank fails, the others are terminated (by their own PIDs) so the job ends instead of hanging
    in a collective."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK='0', MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc if rc >= 0 else 128 - rc


def plan_record(a):
    """--plan-only: this rank's environment and shard of the global batch, exactly as the
    timed run cuts it (no GPU, no collective)."""
    from pdeval import workload as WL
    from pdeval.opcodes import PROBLEM_FORCE_FREE, PROBLEM_KERR
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    pid = PROBLEM_FORCE_FREE if a.problem == 'force_free' else PROBLEM_KERR
    slug = 'force_free' if pid == PROBLEM_FORCE_FREE else 'kerr_magnetosphere'
    wname, ops_all, off_all, _ = load_workload(slug)
    tiled = WL.tiled_indices(len(off_all) - 1, a.n * world, seed=0)
    flops_prog = WL.flops_per_program(pid, ops_all, off_all)
    plan = WL.rank_plan(tiled, world, rank, flops_prog)
    s0, s1 = plan.ranges[rank]
    return {'plan': True, 'rank': rank, 'world': world, 'local_rank': int(os.environ.get('LOCAL_RANK', '0')),
            'master_addr': os.environ.get('MASTER_ADDR'), 'master_port': os.environ.get('MASTER_PORT'),
            'workload': wname, 'total': int(plan.total), 'range': [int(s0), int(s1)], 'n': plan.n,
            'flops': float(flops_prog[plan.idx].sum()), 'flops_total': float(flops_prog[tiled].sum()),
            'idx_head': [int(i) for i in plan.idx[:4]]}


def strict_leg(exprs, device, n=300, seed=0, n_stream=2000):
    """The 'strict' symbolic mode (pdeval.symbolic.suspect + the reference's symbolic stage
    replayed for the grid zeros of those shapes, 60 s per candidate over the SymPy pool) on a
    seed-0 sample of ``n_stream`` depth-4 strings:
    * streaming through the worker pipeline (pdeval.worker.process_batches:
      rows emitted at device rate, suspects resolved asynchronously in the pool): candidates/s
      from the first batch to the last tuple, the suspect fraction and the timeouts;
    * batch-synchronous (the worker's process_batch: one batch, so its slowest replay sets the
      time) on the first ``n`` of them, beside the default mode: its tuples must equal the
      streamed ones of the same rows.
    The whole d4 set's steady-state rate is ``bench.py --strict-full`` (minutes)."""
    import random
    from pdeval.batch import get_validator
    from problems import load_problem
    from problems.force_free.validator import PreciseFoliationValidator
    from pdeval.worker import KnownSolutionTagger, process_batch, process_batches
    strs = [str(e) for e in exprs]
    big = random.Random(seed).sample(strs, min(n_stream, len(strs)))
    sample = big[:n]
    bv = get_validator('force_free', device)
    out = {'sample': len(sample), 'timeout_s': bv.symbolic_timeout}
    t0 = time.perf_counter()
    p = bv.prepare_strings(sample)
    t = bv.finish(p, bv.run_prepared(p), symbolic='off')
    dt = time.perf_counter() - t0
    out['off'] = {'seconds': round(dt, 3), 'candidates_per_s': round(len(sample) / dt, 1),
                  'accepted': int(np.asarray(t['ok']).sum())}
    prob = load_problem('force_free')
    locs = {**prob.unary_ops, **prob.symbols, **prob.constants}
    tagger = KnownSolutionTagger(prob, locs, device)
    v = PreciseFoliationValidator(symbolic='strict')
    kw = {'check_regularity': False, 'fast_point_only': False}
    claimed = [(i + 1, x) for i, x in enumerate(big)]
    stats = {}
    t0 = time.perf_counter()
    got = []
    first = None
    for r in process_batches((claimed[k:k + 4096] for k in range(0, len(claimed), 4096)), v, kw, locs, tagger,
                             stats=stats):
        got.extend(r)
        if first is None:
            first = time.perf_counter() - t0
    dt = time.perf_counter() - t0
    # batch-synchronous strict on the first n rows (compile, device, host steps with every replay)
    t1 = time.perf_counter()
    sync = process_batch(claimed[:len(sample)], v, kw, locs, tagger)
    dts = time.perf_counter() - t1
    out['strict'] = {'seconds': round(dts, 3), 'candidates_per_s': round(len(sample) / dts, 1),
                     'accepted': sum(1 for x in sync if x[1])}
    ids = {i for i, _ in claimed[:len(sample)]}
    same = sorted(x for x in got if x[5] in ids) == sorted(sync)
    out['stream'] = {'sample': len(big), 'batch': 4096, 'seconds': round(dt, 3), 'rows': len(got),
                     'candidates_per_s': round(len(big) / dt, 1), 'first_tuples_s': round(first or 0.0, 3),
                     **stats, 'suspect_fraction': round(stats.get('suspect', 0) / max(1, len(big)), 4),
                     'suspect_fraction_of_grid_zeros': round(stats.get('suspect', 0) / max(1, stats.get('grid_zero', 0)), 4),
                     'tuples_identical_to_batch_strict': same,
                     'note': f'tuple equality checked on the first {len(sample)} rows'}
    out['value_strict'] = out['stream']['candidates_per_s'] if same and len(got) == len(big) else None
    out['value_strict_batch_sync'] = out['strict']['candidates_per_s']
    return out


def strict_full(batch=4096, part=0, parts=1):
    """The streaming 'strict' mode over all 142,004 validated depth-4 strings
    through the worker pipeline (pdeval.worker.process_batches, the default queue batch): rows at
    device rate, suspects replayed in the SymPy pool under the 60 s bound.  Reports the whole
    run's rate, the rate over the rows emitted before the last batch left the device (the
    steady state, before the tail of replays still in the pool), the suspect fraction and the
    timeouts, and whether the final tuples equal the default mode's except on replayed rows."""
    from pdeval.workload import load_programs
    from problems import load_problem
    from problems.force_free.validator import PreciseFoliationValidator
    from pdeval.worker import KnownSolutionTagger, filtered_kwargs, process_batches
    _, _, exprs = load_programs('force_free_d4_validated.npz')
    strs = [str(e) for e in exprs]
    # --parts: a contiguous share of the set per call (one GPU call is bounded in time); the
    # parts' rows and seconds add up to the whole set's rate
    lo, hi = len(strs) * part // parts, len(strs) * (part + 1) // parts
    prob = load_problem('force_free')
    locs = {**prob.unary_ops, **prob.symbols, **prob.constants}
    tagger = KnownSolutionTagger(prob, locs)
    items = [(i + 1, x) for i, x in enumerate(strs)][lo:hi]
    v = PreciseFoliationValidator(symbolic='strict')
    kw = filtered_kwargs(prob.validator)
    stats, got, marks = {}, [], []
    with heartbeat(f"streaming strict mode over {len(items)} strings"):
        t0 = time.perf_counter()
        for r in process_batches((items[k:k + batch] for k in range(0, len(items), batch)), v, kw, locs, tagger,
                                 stats=stats):
            got.extend(r)
            marks.append((time.perf_counter() - t0, len(got)))
        dt = time.perf_counter() - t0
    # the default mode's tuples of the same stream, for the comparison
    off = {t[5]: t for r in process_batches((items[k:k + batch] for k in range(0, len(items), batch)),
                                            prob.validator, kw, locs, tagger) for t in r}
    by = {t[5]: t for t in got}
    changed = sorted(i for i in by if by[i][1] != off[i][1])
    ids = [i for i, _ in items]
    # steady state: the rows out by the time the device stream ended (the first mark at which
    # every batch's ready rows are out), over that time
    n_ready = len(items) - stats.get('sent', 0)
    t_ready = next((t for t, k in marks if k >= n_ready), dt)
    return {'metric': "strict-mode candidates/s (force-free depth-4, worker pipeline, streaming)",
            'part': part, 'parts': parts, 'rows_range': [lo, hi],
            'strings': len(items), 'rows': len(got), 'complete': sorted(by) == ids,
            'seconds': round(dt, 2), 'candidates_per_s': round(len(items) / dt, 1),
            'steady_state_candidates_per_s': round(n_ready / t_ready, 1), 'ready_rows_out_s': round(t_ready, 2),
            **stats, 'suspect_fraction': round(stats.get('suspect', 0) / len(items), 5),
            'suspect_fraction_of_grid_zeros': round(stats.get('suspect', 0) / max(1, stats.get('grid_zero', 0)), 4),
            'verdicts_changed_vs_default': len(changed), 'changed_rows_sample': [dict(items)[i] for i in changed[:20]],
            'batch': batch, 'timeout_s': v.symbolic_timeout}


def worker_throughput(exprs, batch=4096, pipe_batch=32768, inline_n=2000):
    """The drop-in paths over every validated d4 string (the reference's worker protocol,
    general_method_paper_reproduction.py:1756-1816, queue tuples in -> result tuples out):
    * process_batch, one queue-sized batch at a time (native compile, one device call,
      vectorized reasons, known-solution tags);
    * process_batches, the worker loop's four-stage pipeline (later batches compile on host
      threads while batch k+2 is on the device, batch k+1 gets its host steps and batch k
      its tags and tuples), at the
      default queue batch and at larger ones -- its result tuples must equal process_batch's;
    * the inline path: one validate(sympify(s)) per candidate, as the driver's sequential loop
      calls it (:1299-1316), on a seeded sample."""
    import random
    import sympy as sp
    from problems import load_problem
    from pdeval.native import host_threads
    from pdeval.worker import KnownSolutionTagger, filtered_kwargs, process_batch, process_batches
    prob = load_problem('force_free')
    locs = {**prob.unary_ops, **prob.symbols, **prob.constants}
    tagger = KnownSolutionTagger(prob, locs)
    kw = filtered_kwargs(prob.validator)
    items = [(i + 1, str(s)) for i, s in enumerate(exprs)]
    process_batch(items[:batch], prob.validator, kw, locs, tagger)      # warm
    out = {'candidates': len(items), 'host_threads': host_threads()}
    t0 = time.perf_counter()
    ref, ref_batches = [], []
    for k in range(0, len(items), batch):
        ref_batches.append(process_batch(items[k:k + batch], prob.validator, kw, locs, tagger))
        ref.extend(ref_batches[-1])
    dt = time.perf_counter() - t0
    out['process_batch'] = {'batch': batch, 'seconds': round(dt, 3), 'candidates_per_s': round(len(items) / dt),
                            'valid': sum(1 for t in ref if t[1]), 'paper_tagged': sum(1 for t in ref if t[3])}
    for b in (batch, pipe_batch // 2, pipe_batch):
        t0 = time.perf_counter()
        got = []
        for r in process_batches((items[k:k + b] for k in range(0, len(items), b)), prob.validator, kw, locs,
                                 tagger):
            got.extend(r)
        dt = time.perf_counter() - t0
        out[f'pipelined_b{b}'] = {'seconds': round(dt, 3), 'candidates_per_s': round(len(items) / dt),
                                  'tuples_identical': got == ref}
    for procs in (2, 3, 4):
        out[f'pool{procs}_b{batch}'] = worker_pool(ref_batches, len(items), batch, procs)
    sample = random.Random(0).sample(items, min(inline_n, len(items)))
    v = prob.validator
    t_parse = t_val = 0.0
    n_ok = 0
    for _, s in sample:
        t0 = time.perf_counter()
        u = sp.sympify(s, locals=locs)          # the driver's parse (:1257), before validate
        t1 = time.perf_counter()
        ok, _ = v.validate(u, **kw)
        t_val += time.perf_counter() - t1
        t_parse += t1 - t0
        n_ok += bool(ok)
    dt = t_parse + t_val
    out['inline_validate'] = {'sample': len(sample), 'seconds': round(dt, 3),
                              'candidates_per_s': round(len(sample) / dt), 'valid': n_ok,
                              'validate_only_per_s': round(len(sample) / t_val),
                              'us_per_call': {'driver_sympify': round(1e6 * t_parse / len(sample), 1),
                                              'validate': round(1e6 * t_val / len(sample), 1)},
                              'validate_split_us': inline_split(v, sample[:500], locs)}
    # headline: the worker's default queue batch (validator_worker batch_size=4096); the
    # larger batches are detail.  Every pipelined run must give process_batch's tuples.
    out['tuples_identical_all'] = all(out[k]['tuples_identical'] for k in out
                                      if k.startswith('pipelined') or k.startswith('pool'))
    # headline: the worker pool as the reference deploys it (--validators N processes), two
    # processes on this one GPU at the queue's default batch, each taking every other batch;
    # one process's pipeline (pipelined_b4096) and the larger batches are detail
    out['headline_batch'] = batch
    out['headline'] = f'pool2_b{batch}'
    out['candidates_per_s'] = out[out['headline']]['candidates_per_s'] if out['tuples_identical_all'] else None
    out['single_process_candidates_per_s'] = out[f'pipelined_b{batch}']['candidates_per_s']
    return out


def worker_pool(ref_batches, n_items, batch, procs, passes=3):
    """N worker processes on one GPU (scripts/worker_child.py), the reference's --validators N
    (general_method_paper_reproduction.py:802-823): each takes every N-th queue batch of the
    same stream and runs process_batches; started as child processes (no exec in this one),
    timed from a common start line to the last result.  Each process goes over its share
    ``passes`` times (a worker drains a continuous queue: its pipeline fills once, which on one
    142,004-row pass is a tenth of the time).  Their result tuples are compared with
    process_batch's, batch by batch (SHA-256 of each process's tuples in its own order)."""
    import hashlib
    import subprocess
    script = os.path.join(ROOT, 'scripts', 'worker_child.py')
    ps = [subprocess.Popen([sys.executable, script, '--part', str(k), '--parts', str(procs), '--batch', str(batch),
                            '--passes', str(passes)],
                           stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True) for k in range(procs)]
    try:
        for p in ps:
            line = p.stdout.readline()
            while line and line.strip() != 'READY':
                line = p.stdout.readline()
            if not line:
                raise RuntimeError('worker_child exited before READY')
        t0 = time.perf_counter()
        for p in ps:
            p.stdin.write('go\n')
            p.stdin.flush()
        res = [json.loads(p.stdout.readline()) for p in ps]
        wall_parent = time.perf_counter() - t0
        # the timed region: the first process's start to the last one's end (their own
        # perf_counter stamps, one monotonic clock), not the parent's wait, which also holds
        # the children's after-the-fact digests of their tuples and the pipe round trips
        wall = max(r['t1'] for r in res) - min(r['t0'] for r in res)
        for p in ps:
            p.wait(timeout=120)
    finally:
        for p in ps:
            if p.poll() is None:
                p.kill()
    same = True
    for k, r in enumerate(res):
        h = hashlib.sha256()
        for rb in ref_batches[k::procs] * passes:
            h.update(repr(rb).encode())
        same = same and h.hexdigest() == r['digest']
    rows = sum(r['rows'] for r in res)
    return {'processes': procs, 'passes': passes, 'rows': rows, 'seconds': round(wall, 3),
            'candidates_per_s': round(rows / wall) if rows == n_items * passes else None,
            'per_process_s': [round(r['seconds'], 3) for r in res], 'parent_wait_s': round(wall_parent, 3),
            'tuples_identical': same}


def inline_split(v, sample, locs):
    """Where one validate(u) call's time goes (force-free plugin): the canonical tree, the
    compile (flatten.py), the device call (pdeval_validate_batch: upload, launch chain or its
    captured graph, download, sync) and the host steps + reason."""
    import sympy as sp
    from pdeval import problem_defs as P
    bv = v._validator()
    pd = P.get('force_free')
    t = {'canon': 0.0, 'compile': 0.0, 'device': 0.0, 'host': 0.0}
    for _, s in sample:
        u0 = sp.sympify(s, locals=locs)
        t0 = time.perf_counter()
        u = v._canon(u0)
        t1 = time.perf_counter()
        ops, off, notes = P.compile_exprs(pd, [u])
        t2 = time.perf_counter()
        r = bv.run(ops, off)
        t3 = time.perf_counter()
        bv.table(bv.host_steps(r, ops, off, [u]), ops, off, notes)
        t4 = time.perf_counter()
        for k, a, b in (('canon', t0, t1), ('compile', t1, t2), ('device', t2, t3), ('host', t3, t4)):
            t[k] += b - a
    return {k: round(1e6 * x / len(sample), 1) for k, x in t.items()}


def cpu_baseline_sympy(procs, budget_s):
    """The SymPy CPU path (oracle/sympy_validator.py, the reference's validate restated) on
    the host cores, 60 s per-candidate timeout, in two legs of the wall budget: C1 (the 111
    depth<=2 candidates that reach validate, 25 %) and a seed-0 sample of 1,000 depth-4
    candidates (75 %: 90 s by default, so that candidates started in the first 30 s can reach
    the 60 s timeout and the rate counting timeouts differs from the rate without them).
    value = the depth-4 rate (the bench's workload), counting completed candidates; the C1
    rate and the rates counting timeouts are in detail.  The restatement's
    per-candidate time against the reference's own validate, measured on 200 depth-4
    candidates in the build container (oracle/calibrate_sympy.py), is reported beside it."""
    import gzip
    import random
    sys.path.insert(0, os.path.join(ROOT, 'oracle'))
    import sympy_bench
    with gzip.open(os.path.join(ROOT, 'tests', 'golden', 'streams', 'force_free_d3_validated.txt.gz'), 'rt') as f:
        c1 = [l.rstrip('\n').split('\t')[-1] for l in f if int(l.split('\t')[-2]) <= 2]
    with gzip.open(os.path.join(ROOT, 'tests', 'golden', 'streams', 'force_free_d4_validated.txt.gz'), 'rt') as f:
        d4 = [l.rstrip('\n').split('\t')[-1] for l in f]
    d4s = random.Random(0).sample(d4, 1000)
    r_c1 = sympy_bench.run(c1, procs, timeout=60, budget_s=0.25 * budget_s)
    r_d4 = sympy_bench.run(d4s, procs, timeout=60, budget_s=0.75 * budget_s)
    cal = None
    cp = os.path.join(ROOT, 'profiles', 'r03_sympy_calibration.json')
    if os.path.exists(cp):
        with open(cp) as f:
            c = json.load(f)
        cal = {k: c[k] for k in ('restatement_vs_reference_time_ratio', 'completed_both', 'verdicts_agree',
                                 'timeouts', 'median_s', 'sample') if k in c}
    return {'value': r_d4['rate_completed'], 'unit': 'candidates/s', 'cores': procs, 'kind': 'port',
            'sample': (f"SymPy restatement of the reference's validate (oracle/sympy_validator.py), "
                       f"multiprocessing.Pool({procs}), 60 s per-candidate timeout: a seed-0 sample of "
                       f"1,000 depth-4 candidates ({0.75 * budget_s:.0f} s wall budget; value), and C1 "
                       f"({len(c1)} depth<=2 candidates, {0.25 * budget_s:.0f} s)"),
            'timeouts_note': ('the d4 leg observed timeouts' if r_d4['timeouts_60s'] else
                              'no sampled depth-4 candidate reached the 60 s timeout within the budget'),
            'rate_d4': r_d4['rate_completed'], 'rate_d4_incl_timeouts': r_d4['rate_incl_timeouts'],
            'rate_c1': r_c1['rate_completed'], 'rate_c1_incl_timeouts': r_c1['rate_incl_timeouts'],
            'calibration': cal, 'detail': {'d4': r_d4, 'c1': r_c1}}


def cpu_baseline(pid, ops_all, off_all, idx, budget_s):
    """The C oracle (a CPU port of the same validation) on a bounded sample of the same
    workload, one core."""
    import oracle_lib as O
    sample = idx[:4096]
    from pdeval.workload import gather_programs
    ops, off = gather_programs(ops_all, off_all, sample)
    done, t0 = 0, time.perf_counter()
    while done < len(sample) and time.perf_counter() - t0 < budget_s:
        O.validate(pid, ops, off, first=done, count=64)
        done += 64
    dt = time.perf_counter() - t0
    return {'value': done / dt, 'unit': 'candidates/s', 'cores': 1, 'kind': 'port',
            'sample': f'first {done} candidates of this batch (same 4097 points each, full grid), '
                      f'C oracle oracle/jet_oracle.c, 1 thread, {dt:.1f}s'}


if __name__ == '__main__':
    main()
