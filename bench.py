#!/usr/bin/env python3
"""bench.py — MI355X path-tracing integrator benchmark (driver contract).

Metric (BASELINE.json): Msamples/s (+ achieved HBM GB/s) on vol2_final_scene
800x800 at 1/2/4/8 MI355X. One sample = one camera path for one pixel
(renderer.py:453-471 prints the same quantity as "M pix/s" at 1 spp/launch).

Workload (BASELINE.json configs[1]): vol2_final_scene 800x800, megakernel
integrator, 64 spp per step; --steps 16 steps by default, i.e. 1024 spp per
GPU, the sample count of the north-star target (configs[2]; --variant wf runs
that config's wavefront integrator). A "step" is one call of the hot path
over the whole image for spp-per-step samples. Scene = the reference's own
vol2_final_scene compiled arrays captured at random.seed(1234)
(tests/golden/vol2_final_scene.npz), camera from the reference's camera math.

Multi-GPU (python3 bench.py --gpus N, or python -m torch.distributed.run ...
bench.py --gpus N): one process per GPU; without a launcher's RANK in the
environment bench.py starts the N ranks itself (ptmi.launch). By default the image is tile-sharded (BASELINE.json
configs[4]): rank r renders the interleaved row bands it owns for every sample
of every step, so the total workload (W x H x spp_per_step x steps) is fixed
and N GPUs split it (strong scaling); the bands' height is chosen so every
rank owns the same number of rows. One RCCL gather of each rank's owned rows
onto rank 0, inside the timed region, assembles the image
(ptmi.distributed.assemble_image), which is bit-identical to the 1-GPU render. value = total samples / max-over-ranks
wall time. --shard samples keeps the weak-scaling alternative (every rank the
whole image, disjoint sample indices).

Rank 0 at N=1 also times the CPU oracle (oracle/, a C restatement of the
reference's kernels.py: the reference's ti.cpu path cannot run here, Taichi is
absent) on a bounded slice of the same workload, and reports the dominant
kernel's roofline from HIP events recorded around its launches in the timed
region: per-launch time = the union of the launches' [start, end] intervals
divided by the launch count, because consecutive megakernel calls are
pipelined on two streams and overlap (tools/trace_busy.py computes the same
figure from a rocprofv3 kernel trace). `roofline.traffic` (PMC HBM-side bytes per launch, profiles/traffic.json)
and `valu_diagnostic` (VALU issue share, lane efficiency and wave wait share of
the dominant kernel, profiles/valu.json) come from committed rocprofv3 passes
over the same workload (tools/pmc_traffic.py, tools/pmc_valu.py).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'path-tracer-python_amd'))

METRIC = 'Msamples/s + achieved HBM GB/s, vol2_final_scene 800x800 at 1/2/4/8 MI355X'
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
BG = {'vol2_final_scene': (0.0, 0.0, 0.0), 'vol2_final_scene_comparison': (0.0, 0.0, 0.0),
      'wavefront_comparison': (0.7, 0.8, 1.0), 'cornell_smoke': (0.0, 0.0, 0.0)}
# BASELINE.json configs as bench presets: (scene, width, integrator, spp per step, steps)
PRESETS = {
    'c2': ('vol2_final_scene', 800, 'mk', 64, 16),       # configs[1]; 16 steps = the 1024-spp north star
    'c3': ('vol2_final_scene', 800, 'wf', 64, 16),       # configs[2]: wavefront, 1024 spp
    'c4': ('cornell_mesh_fog', 1024, 'mk', 32, 16),      # configs[3]: OBJ mesh + fog, 512 spp
    'c5': ('vol2_final_scene_comparison', 3840, 'mk', 16, 256),  # configs[4]: 4K @ 4096 spp, tile-sharded
}

# Algorithmic HBM bytes per unit (DESIGN.md "Roofline"): what each kernel must
# move at minimum for one unit of work in the queue layout of pt_wavefront.hip.
ALGO_BYTES = {
    # read o,d (24 B) + write hit t,ref (8 B) per ray
    'wf_intersect': ('rays', 32),
    # per traced segment that continues: read list index 4 B + hit 8 B + ray
    # record 48 B, write the next record 48 B (surface shading and medium alike)
    'wf_scatter': ('rays', 108),
    # SURVEY.md §8d graded figure per sample, B_sample = 44 + 24 + 128*S with
    # S = measured segments/sample: the bytes the reference's stage pipeline
    # must move for one camera path (the megakernel keeps them in registers)
    'megakernel': ('samples', None),
    # initial slot state (item word) per slot
    'wf_generate': ('rays', 4),
    # a batch's tail, every remaining path in one launch: per segment the
    # intersect and scatter figures together (32 + 108 B)
    'wf_drain': ('rays', 140),
    # accumulator read + write 24 B + batch x 12 B staging read, per pixel
    'wf_resolve': ('pixels', 24),
    # accumulator read + write 24 B + batch x 12 B staging read, per pixel
    'mk_resolve': ('pixels', 24),
}


def kernel_units(kernel, segments, tail, samples, pixels, prof):
    """Units of work ``kernel`` processed in the timed steps (the unit of
    ALGO_BYTES[kernel]): the wavefront's segments traced by its tail launch
    (device counter [5], `tail`) are wf_drain's, the rest wf_intersect's and
    wf_scatter's; a resolve's unit is a pixel per launch."""
    return {'wf_intersect': segments - tail, 'wf_scatter': segments - tail, 'megakernel': samples,
            'wf_generate': 0, 'wf_drain': tail,
            'wf_resolve': pixels * prof.get('wf_resolve', {}).get('launches', 0),
            'mk_resolve': pixels * prof.get('mk_resolve', {}).get('launches', 0)}[kernel]


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument('--gpus', type=int, default=int(os.environ.get('WORLD_SIZE', '1')))
    p.add_argument('--preset', choices=sorted(PRESETS), default='c2',
                   help='BASELINE config; --scene/--width/--variant/--spp-per-step/--steps override it')
    p.add_argument('--steps', type=int, default=None)
    p.add_argument('--warmup', type=int, default=2)
    p.add_argument('--spp-per-step', type=int, default=None)
    p.add_argument('--variant', choices=('wf', 'mk'), default=None)
    p.add_argument('--scene', default=None)
    p.add_argument('--width', type=int, default=None)
    p.add_argument('--max-depth', type=int, default=50)
    p.add_argument('--seed', type=int, default=0)
    p.add_argument('--cpu-seconds', type=float, default=12.0)
    p.add_argument('--no-cpu-baseline', action='store_true')
    p.add_argument('--save-image', default='')
    p.add_argument('--save-accum', default='',
                   help='rank 0 writes the assembled float32 accumulator (H, W, 3) to this .npy file')
    p.add_argument('--launch-timeout', type=float, default=3600.0,
                   help='--gpus N > 1 without a launcher: seconds the ranks may run before they are stopped')
    p.add_argument('--dist-backend', choices=('nccl', 'gloo'), default=None,
                   help='nccl = RCCL over xGMI (the product path, the default for --gpus > 1); gloo only to '
                        'rehearse the multi-rank flow with several ranks on one GPU (host-side collective). '
                        'Given explicitly with --gpus 1, the process group is created at world size 1 and '
                        'every collective of the N-GPU flow runs (gather, all-reduce MAX, all-gather)'),
    p.add_argument('--no-overlap', action='store_true',
                   help='megakernel: each step waits for the previous one to finish (default: consecutive '
                        'steps overlap, Integrator.render_mk_overlapped)')
    p.add_argument('--traversal', choices=('stack', 'stackless'), default='stack',
                   help="BVH traversal: the reference's default stack walk (traverse_bvh_legacy, kernels.py:625) "
                        'or its USE_STACKLESS_TRAVERSAL walk (traverse_bvh_stackless, kernels.py:453)')
    p.add_argument('--shard', choices=('samples', 'tiles'), default='tiles',
                   help='multi-GPU partition: row-band tiles of a fixed total workload (strong scaling, default; '
                        'bit-identical to 1 GPU) or disjoint sample shards of the whole image (weak scaling)')
    a = p.parse_args(argv)
    scene, width, variant, sps, steps = PRESETS[a.preset]
    a.scene = a.scene or scene
    a.width = a.width or width
    a.variant = a.variant or variant
    a.spp_per_step = a.spp_per_step or sps
    a.steps = a.steps or steps
    a.process_group = a.gpus > 1 or a.dist_backend is not None
    a.dist_backend = a.dist_backend or 'nccl'
    return a


def load_workload(scene, width):
    """(SceneArrays, camera upload dict, background, data note) of a workload:
    the reference's own compiled arrays (tests/golden fixture) where captured,
    else the scene built by ptmi.scenes at random.seed(1234) and compiled here
    (compile_scene + native SAH builder)."""
    from ptmi import scene_data as sd
    import numpy as np
    path = os.path.join(sd.golden_dir(), scene + '.npz')
    if os.path.exists(path) and f'cam{width}_center' in np.load(path).files:
        return (sd.load_fixture(scene), sd.fixture_camera(scene, width), BG[scene],
                f'reference scene {scene} compiled at random.seed(1234) (tests/golden fixture); no external dataset')
    import random
    from ptmi import scenes
    random.seed(1234)
    sc = scenes.SCENES[scene]()
    sc.cam.img_width = width
    sc.cam.initialize()
    sa = sd.compile_world(sc.world)
    return (sa, sd.camera_upload(sc.cam), tuple(sc.background),
            f'{scene} built by ptmi.scenes at random.seed(1234) (build-supplied scene; OBJ asset in-tree); '
            'no external dataset')


def cpu_info():
    """CPU model and core counts of this host: the model from /proc/cpuinfo,
    os.cpu_count() (every CPU of the machine) and the CPUs this process may
    run on (sched_getaffinity)."""
    model = None
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    model = line.split(':', 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        allowed = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        allowed = os.cpu_count() or 1
    return {'cpu_model': model, 'os_cpu_count': os.cpu_count(), 'affinity_cpus': allowed}


def cpu_baseline(sa, cam, bg, scene, variant, max_depth, seed, budget_s):
    """Time the CPU oracle on a bounded sample of the workload (rank 0, N=1):
    the whole frame (every pixel, so the sample has the workload's mix of sky,
    fog and geometry) at as many samples per pixel as fit the time budget,
    after a 1-spp whole-frame calibration pass. Threads: OMP_NUM_THREADS when
    set (the GPU box sets it to the CPU share of one GPU, 16), else every CPU
    this process may run on."""
    import numpy as np
    import oracle
    W, H = cam['width'], cam['height']
    info = cpu_info()
    env = os.environ.get('OMP_NUM_THREADS')
    threads = int(env) if env and env.isdigit() and int(env) > 0 else info['affinity_cpus']
    osc = oracle.OracleScene(sa)
    fr = oracle.make_frame(cam, bg, max_depth, seed, W, H)
    acc = np.zeros((H, W, 3), np.float32)
    t = time.perf_counter()
    oracle.render(osc, fr, variant, acc, (0, 0, W, H), 0, 1, threads)
    t1 = time.perf_counter() - t
    spp = max(1, int(budget_s / max(t1, 1e-3)))
    t = time.perf_counter()
    oracle.render(osc, fr, variant, acc, (0, 0, W, H), 1, spp, threads)
    dt = time.perf_counter() - t
    n = W * H * spp
    return {'value': round(n / dt / 1e6, 4), 'unit': 'Msamples/s', 'cores': threads, 'kind': 'port',
            'threads_source': 'OMP_NUM_THREADS' if env else 'sched_getaffinity', **info,
            'sample': f'{scene} {W}x{H}, the whole frame x {spp} spp (samples 1..{spp}, after a 1-spp '
                      f'calibration pass), {"wavefront" if variant == "wf" else "megakernel"} semantics, C oracle '
                      f'(restatement of kernels.py; Taichi ti.cpu absent), {threads} OpenMP threads, {dt:.1f} s'}


TRAFFIC_FILE = os.path.join(ROOT, 'profiles', 'traffic.json')


VALU_FILE = os.path.join(ROOT, 'profiles', 'valu.json')


def valu_diagnostic(a, kernel):
    """Secondary compute-side diagnostic of the dominant kernel
    from the committed PMC passes (tools/pmc_valu.py), when collected on this
    scene/integrator; None otherwise."""
    try:
        with open(VALU_FILE) as f:
            rows = json.load(f)
    except (OSError, ValueError):
        return None
    return rows.get(f'{a.scene}:{a.width}:{a.variant}:{kernel}')


def measured_traffic(a, kernel):
    """HBM-side bytes per launch of ``kernel`` from the committed PMC summary
    (tools/pmc_traffic.py: FETCH_SIZE x 2 + WRITE_SIZE per dispatch, gfx950
    correction of MI355X_MICROARCH.md "HBM"), when it was collected on this
    exact workload; None otherwise."""
    try:
        with open(TRAFFIC_FILE) as f:
            rows = json.load(f)
    except (OSError, ValueError):
        return None
    key = f'{a.scene}:{a.width}:{a.variant}:{a.spp_per_step}:{a.max_depth}:{kernel}'
    r = rows.get(key)
    if not r:
        return None
    return {'bytes_per_launch': r['bytes_per_launch'], 'source': r['source']}


class BenchRun:
    """The hot-path call shape of one bench rank: workload, device scene,
    frame (this rank's bands), and one step = one render call of
    spp_per_step samples. tests/test_gpu_bench_shapes.py drives this same
    object to check the benchmarked calls against the oracle."""

    def __init__(self, a, dev, rank=0, world=1):
        from ptmi import device
        from ptmi.distributed import Shard
        self.a = a
        self.sa, self.cam, self.bg, self.data_note = load_workload(a.scene, a.width)
        self.W, self.H = self.cam['width'], self.cam['height']
        self.integ = device.Integrator(device.DeviceScene(self.sa, dev))
        self.shard = Shard.balanced(rank, world, a.shard, self.H)
        self.frame = device.make_frame(self.cam, self.bg, a.max_depth, a.seed, self.W, self.H,
                                       band=self.shard.band(), traversal=a.traversal)
        self.sps = a.spp_per_step
        self.rows = len(self.shard.rows(self.H))

    def sample_base(self, step):
        return self.shard.sample_range(step, self.sps)[0]

    def render(self, acc, s0, n):
        if self.a.variant == 'mk':
            self.integ.render_mk(self.frame, acc, s0, n, overlap=not self.a.no_overlap)
        else:
            self.integ.render_wf(self.frame, acc, s0, n)

    def step(self, acc, k):
        """Step k: samples [sample_base(k), sample_base(k) + spp_per_step) of this rank's rows."""
        self.render(acc, self.sample_base(k), self.sps)


def describe(a, W, H, world, shard):
    """Workload description of the JSON line: (total spp, scaling, config)."""
    total_spp = a.spp_per_step * a.steps * (world if a.shard == 'samples' else 1)
    rows_rank = len(shard.rows(H))
    cfg = {
        'workload': f'{a.scene} {W}x{H} @ {total_spp} spp in total ({a.steps} steps x {a.spp_per_step} spp'
                    f'{" x " + str(world) + " sample shards" if a.shard == "samples" and world > 1 else ""}), '
                    f'{"wavefront" if a.variant == "wf" else "megakernel"} integrator, max_depth {a.max_depth}',
        'scene': a.scene, 'width': W, 'height': H, 'variant': a.variant, 'traversal': a.traversal,
        'spp_per_step': a.spp_per_step, 'total_spp': total_spp,
        'partition': a.shard,
        'band_rows': shard.band()[0] if a.shard == 'tiles' and world > 1 else None,
        'rows_per_rank': rows_rank,
        'max_depth': a.max_depth, 'seed': a.seed,
        'parallelism': (f'{a.shard}-shard x{world} + {"RCCL" if a.dist_backend == "nccl" else "gloo"} '
                        f'{"gather of owned row bands" if a.shard == "tiles" else "sum-reduce"}'
                        if world > 1 else 'single GPU'),
    }
    return total_spp, ('weak' if a.shard == 'samples' else 'strong'), cfg


def throughput(samples_all, elapsed_max_s):
    """`value` of the JSON line: every rank's samples / the slowest rank's
    wall time (max over ranks, barrier-bracketed), in Msamples/s."""
    return samples_all / elapsed_max_s / 1e6


def gather_ranks(vals, dev, world=None):
    """Per-rank float rows (one all_gather, ptmi.distributed.gather_ranks) ->
    list of lists; [vals] without a process group."""
    from ptmi.distributed import gather_ranks as _gather
    return _gather(vals, dev)


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def main():
    a = parse()
    if a.gpus > 1 and 'RANK' not in os.environ:
        # `python3 bench.py --gpus N` with no launcher: start the N ranks here
        # (ptmi.launch), before anything in this process touches the GPU, and
        # exit with the first failing rank's code; rank 0 prints the line
        from ptmi.launch import launch_ranks
        sys.exit(launch_ranks([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], a.gpus,
                              timeout_s=a.launch_timeout))
    import torch
    import torch.distributed as dist
    from ptmi import _lib
    from ptmi.distributed import assemble_image, max_over_ranks

    world = a.gpus
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    # one process per GPU; the gloo rehearsal may put several ranks on one device
    dev_index = local_rank if a.dist_backend == 'nccl' else local_rank % max(1, torch.cuda.device_count())
    dev = torch.device('cuda', dev_index)
    pg = a.process_group  # --gpus > 1, or an explicit --dist-backend at --gpus 1
    if pg:
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        if 'RANK' not in os.environ:  # a plain `python bench.py --gpus 1 --dist-backend nccl`
            os.environ.update(RANK='0', WORLD_SIZE='1', MASTER_PORT=os.environ.get('MASTER_PORT', str(_free_port())))
        torch.cuda.set_device(dev)
        if a.dist_backend == 'nccl':
            dist.init_process_group('nccl', device_id=dev)
        else:
            dist.init_process_group('gloo')
        if dist.get_world_size() != world:
            sys.exit(f'--gpus {world} but torch.distributed has {dist.get_world_size()} ranks')
    world_size = dist.get_world_size() if pg else 1

    run = BenchRun(a, dev, rank, world)
    integ, frame, sa, cam, bg = run.integ, run.frame, run.sa, run.cam, run.bg
    W, H, sps = run.W, run.H, run.sps
    data_note = run.data_note
    shard = run.shard
    acc = torch.zeros((H, W, 3), dtype=torch.float32, device=dev)

    for k in range(a.warmup):
        run.step(acc, k)
    # warm the collective too: RCCL sets up a collective's channels on its
    # first call, which must not land in the timed region
    assemble_image(acc, shard, dst=0)
    torch.cuda.synchronize(dev)
    acc.zero_()  # all rows: the warm-up gather left other ranks' bands on the root
    integ.reset_counters()
    torch.cuda.synchronize(dev)
    if pg:
        dist.barrier()

    # Per-kernel durations (roofline): HIP events around every launch, on the
    # stream it runs on. The megakernel (2 events per 18-ms launch) is timed
    # inside the timed region. The wavefront's pipes are concurrent streams and
    # an event per launch costs them ~10 %, so its kernels are timed in a
    # second pass over the same K steps into a scratch accumulator and the
    # timed region runs without events.
    inline = a.variant == 'mk'
    with _lib.KernelTimer(max_launches=100_000 if inline else 0) as kt:
        torch.cuda.synchronize(dev)
        if pg:
            dist.barrier()
        t0 = time.perf_counter()
        for k in range(a.steps):
            run.step(acc, a.warmup + k)
        t_render_end = None
        if pg:
            torch.cuda.synchronize(dev)  # this rank's own render time (per-rank balance), then the gather
            t_render_end = time.perf_counter()
        assemble_image(acc, shard, dst=0)
        torch.cuda.synchronize(dev)
        if pg:
            dist.barrier()
        elapsed_rank = time.perf_counter() - t0
    render_rank = (t_render_end - t0) if t_render_end is not None else elapsed_rank
    elapsed = max_over_ranks(elapsed_rank, dev if a.dist_backend == 'nccl' else None)
    cnt = integ.read_counters()
    if not inline:
        acc_k = torch.zeros_like(acc)
        with _lib.KernelTimer(max_launches=100_000) as kt:
            for k in range(a.steps):
                run.step(acc_k, a.warmup + k)
            torch.cuda.synchronize(dev)
        del acc_k
    rows_rank = run.rows
    samples_rank = W * rows_rank * sps * a.steps
    samples_all = samples_rank * world if a.shard == 'samples' else W * H * sps * a.steps
    value = throughput(samples_all, elapsed)
    total_spp, scaling, config = describe(a, W, H, world, shard)

    prof = kt.result
    # per-launch GPU time = union of the kind's launch intervals / launches
    # (ptmi_prof_stop_busy): pipelined megakernel calls overlap their
    # neighbours, so each launch's own start->end spans about two steps
    dom = max((k for k in prof if prof[k]['launches']), key=lambda k: prof[k]['busy_ms'])
    S = cnt['segments'] / samples_rank
    M = cnt['medium'] / samples_rank
    b_sample = 44 + 24 + 128 * S  # SURVEY.md §8d whole-pipeline algorithmic bytes per sample
    unit_name, unit_bytes = ALGO_BYTES[dom]
    if unit_bytes is None:
        unit_bytes = b_sample
    # segments traced by the wavefront's tail launch (wf_drain) belong to its
    # time, not to wf_intersect's / wf_scatter's
    tail = (integ.tail_segments() or 0) if a.variant == 'wf' else 0
    units = kernel_units(dom, cnt['segments'], tail, samples_rank, W * rows_rank, prof)
    dom_ms = prof[dom]['busy_ms']
    launches = prof[dom]['launches']
    avg_launch_ms = dom_ms / max(1, launches)
    achieved = units * unit_bytes / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
    # the committed PMC passes were collected on the full frame at one GPU
    traffic = measured_traffic(a, dom) if world == 1 or a.shard == 'samples' else None
    valu = valu_diagnostic(a, dom)
    per_rank = gather_ranks([rank, rows_rank, samples_rank, render_rank, elapsed_rank, dom_ms],
                            dev if a.dist_backend == 'nccl' else 'cpu', world)

    out = {
        'metric': METRIC,
        'value': round(value, 3),
        'unit': 'Msamples/s',
        'n_gpus': world,
        'world_size': world_size,
        'steps': a.steps,
        'warmup': a.warmup,
        'ms_per_step': round(elapsed * 1e3 / a.steps, 4),
        'higher_is_better': True,
        'scaling': scaling,
        'vs_baseline': None,
        'dtype': 'f32',
        'data': data_note,
        'config': config,
        'roofline': {
            'bound': 'hbm', 'kernel': dom,
            'achieved': round(achieved, 3), 'peak': HBM_PEAK_GBPS, 'unit': 'GB/s',
            'frac': round(achieved / HBM_PEAK_GBPS, 6),
            'traffic': traffic['bytes_per_launch'] if traffic else None,
            'traffic_source': traffic['source'] if traffic else None,
            # what the counters say the kernel really moves to/from HBM (incl.
            # Infinity-Cache hits): PMC bytes per launch / busy time per launch
            'measured_GBps': round(traffic['bytes_per_launch'] / (avg_launch_ms * 1e-3) / 1e9, 3)
            if traffic and avg_launch_ms > 0 else None,
            # compute side of the same kernel: VALU issue share x lane efficiency
            # (profiles/valu.json): the fraction of the chip's FP32 lanes doing work
            'compute_frac': round(valu['valu_issue_frac'] * valu['lane_efficiency'], 4) if valu else None,
            'achieved_note': ('achieved = algorithmic bytes (SURVEY.md §8d B_sample model) / busy time; '
                              'it is not HBM traffic: see measured_GBps'),
            'algorithmic_bytes_per_launch': round(units * unit_bytes / max(1, launches), 1),
            'unit_of_work': f'{unit_bytes:.1f} B per {unit_name[:-1] if unit_name.endswith("s") else unit_name}',
            'avg_launch_ms': round(avg_launch_ms, 5),
            'avg_launch_own_ms': round(prof[dom]['ms'] / max(1, launches), 5),
            'launches': launches,
            'timing_truncated': bool(kt.truncated),
            'timing': ('HIP events per launch on its stream, ' +
                       ('in the timed region' if inline else 'in a second pass over the same steps') +
                       "; avg_launch_ms = union of the launches' [start, end] intervals / launches "
                       '(pipelined launches overlap; avg_launch_own_ms = mean start->end of one launch)'),
        },
        'valu_diagnostic': valu,
        'kernels_ms': {k: round(v['ms'], 3) for k, v in prof.items() if v['launches']},
        'kernels_busy_ms': {k: round(v['busy_ms'], 3) for k, v in prof.items() if v['launches']},
        'segments_per_sample': round(S, 4),
        'tail_segments_per_sample': round(tail / samples_rank, 4) if a.variant == 'wf' else None,
        'collectives': ({'backend': dist.get_backend(), 'world_size': world_size,
                         'calls': ['gather (assemble_image, tiles) / reduce (samples)', 'all_reduce MAX (elapsed)',
                                   'all_gather (per-rank rows)']} if pg else None),
        'medium_traversals_per_sample': round(M, 4),
        'pipeline_algorithmic_GBps': round(value * 1e6 * b_sample / 1e9, 3),
        'ranks': [{'rank': int(r[0]), 'rows': int(r[1]), 'samples': int(r[2]), 'render_s': round(r[3], 4),
                   'elapsed_s': round(r[4], 4), 'kernel_busy_ms': round(r[5], 3)} for r in per_rank],
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out['cpu_baseline'] = cpu_baseline(sa, cam, bg, a.scene, a.variant, a.max_depth, a.seed, a.cpu_seconds)
    elif rank == 0:
        out['cpu_baseline'] = None
    if rank == 0:
        if a.save_accum:
            import numpy as np
            np.save(a.save_accum, acc.cpu().numpy())
        if a.save_image:
            from PIL import Image
            # tiles: every pixel has sps * steps samples; samples: each rank added its own
            img = integ.tonemap(acc, total_spp).cpu().numpy()
            Image.fromarray(img).save(a.save_image)
        print(json.dumps(out), flush=True)
    if pg:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
