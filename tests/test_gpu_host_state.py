"""GPU tests of the host-side state around the C-ABI (through the C-ABI, on
the box's GPU):

* two host threads calling ptmi_wf_render on one device at once: each call
  drives all pipes and reads their live counts back, so the per-device
  readback slots must not be shared between calls (a call whose pipe read
  another call's 0 would stop early and drop samples without an error);
* the device a DeviceScene is bound to decides where its launches go, not
  whichever device happens to be current;
* a staged megakernel call whose (tile, sample, pixel) item ids would pass
  2^32 is split into batches instead of failing;
* the profiler's busy time (ptmi_prof_stop_busy, bench.py's per-launch time
  for the roofline) is the union of overlapping launches: pipelined
  megakernel calls overlap, so it is below the summed durations and close to
  the wall time of the calls.
"""
import threading

import numpy as np
import pytest

from parity_helpers import scene_inputs

pytestmark = pytest.mark.gpu


def _frame_acc(cam, win, seed=5):
    import torch
    from ptmi import device
    W, H = cam['width'], cam['height']
    fr = device.make_frame(cam, (0.0, 0.0, 0.0), 50, seed, W, H, win)
    return fr, torch.zeros((H, W, 3), dtype=torch.float32, device='cuda')


def test_wf_render_concurrent_threads_one_device():
    import torch
    from ptmi import device
    sa, cam, _ = scene_inputs('vol2_final_scene', 800)
    win, spp = (352, 352, 96, 96), 6
    dscene = device.DeviceScene.from_arrays(sa)
    n = 3
    integs = [device.Integrator(dscene) for _ in range(n)]
    accs = [_frame_acc(cam, win) for _ in range(n)]
    streams = [torch.cuda.Stream() for _ in range(n)]
    errors = []
    start = threading.Barrier(n)

    def work(k):
        try:
            fr_k, acc_k = accs[k]
            with torch.cuda.stream(streams[k]):
                start.wait()
                for rep in range(2):  # two calls per thread: overlapping starts and ends
                    integs[k].render_wf(fr_k, acc_k, rep * spp, spp, stream=streams[k])
            streams[k].synchronize()
        except Exception as e:  # noqa: BLE001 (reported below)
            errors.append(e)

    threads = [threading.Thread(target=work, args=(k,)) for k in range(n)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    assert not errors, errors
    # each thread made two calls (samples 0..spp-1, then spp..2spp-1): compare
    # with the same two calls made from this thread alone
    ref_integ = device.Integrator(dscene)
    fr2, ref2 = _frame_acc(cam, win)
    ref_integ.render_wf(fr2, ref2, 0, spp)
    ref_integ.render_wf(fr2, ref2, spp, spp)
    torch.cuda.synchronize()
    ref2 = ref2.cpu().numpy()
    assert ref2.sum() > 0
    for k in range(n):
        got = accs[k][1].cpu().numpy()
        assert np.array_equal(got, ref2), f'thread {k}: differs from the single-threaded render'
        paths = integs[k].read_counters()['paths']
        assert paths == 2 * spp * win[2] * win[3], f'thread {k}: {paths} paths'


def test_scene_device_is_fixed_at_construction():
    import torch
    from ptmi import device
    sa, cam, _ = scene_inputs('wavefront_comparison', 400)
    ds = device.DeviceScene.from_arrays(sa, 'cuda')
    assert ds.device.index == torch.cuda.current_device()
    integ = device.Integrator(ds)
    fr, acc = _frame_acc(cam, (100, 60, 64, 48))
    integ.render_mk(fr, acc, 0, 2)
    torch.cuda.synchronize()
    ref = acc.cpu().numpy()
    if torch.cuda.device_count() < 2:
        # one GPU: a foreign-device stream must be refused, not used
        class _Fake:
            device = torch.device('cuda', 1)
            cuda_stream = 0
        with pytest.raises(Exception, match='stream is on'):
            integ.render_mk(fr, acc, 0, 1, stream=_Fake())
        return
    # scene on cuda:1 while cuda:0 is current: the launch must go to cuda:1
    torch.cuda.set_device(0)
    ds1 = device.DeviceScene.from_arrays(sa, 'cuda:1')
    integ1 = device.Integrator(ds1)
    acc1 = torch.zeros_like(acc, device='cuda:1')
    integ1.render_mk(fr, acc1, 0, 2)
    torch.cuda.synchronize('cuda:1')
    assert np.array_equal(acc1.cpu().numpy(), ref)


def test_mk_staged_item_ids_past_2_to_32_split_into_batches():
    import torch
    from edge_scenes import edge_scene
    from ptmi import device
    sa, cam, bg = edge_scene('empty')
    W, H = cam['width'], cam['height']
    integ = device.Integrator(device.DeviceScene.from_arrays(sa))
    fr = device.make_frame(cam, bg, 50, 0, W, H, (0, 0, 1, 1))  # one pixel = one 8x8 tile
    n = (1 << 26) + 3  # 64 * n item ids > 2^32
    acc = torch.zeros((H, W, 3), dtype=torch.float32, device='cuda')
    integ.reset_counters()
    integ.render_mk(fr, acc, 0, n)
    torch.cuda.synchronize()
    assert integ.read_counters()['paths'] == n
    # every sample of the empty scene is bg; the resolve adds them in sample order
    want = np.add.accumulate(np.full(n, np.float32(bg[0]), np.float32))[-1]
    assert acc[0, 0, 0].item() == want
    assert acc[0, 1:].abs().sum().item() == 0.0


def test_prof_busy_time_is_the_union_of_overlapping_launches():
    import time
    import torch
    from ptmi import device, _lib
    sa, cam, _ = scene_inputs('vol2_final_scene', 800)
    integ = device.Integrator(device.DeviceScene.from_arrays(sa))
    fr, acc = _frame_acc(cam, (0, 0, cam['width'], cam['height']))
    integ.render_mk(fr, acc, 0, 4, overlap=True)  # warm-up: workspaces, streams
    torch.cuda.synchronize()
    n, spp = 6, 8
    with _lib.KernelTimer(max_launches=1000) as kt:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(n):
            integ.render_mk(fr, acc, 4 + k * spp, spp, overlap=True)
        torch.cuda.synchronize()
        wall_ms = (time.perf_counter() - t0) * 1e3
    mk = kt.result['megakernel']
    assert mk['launches'] == n and not kt.truncated
    assert 0.0 < mk['busy_ms'] <= mk['ms'] + 1e-3   # a union never exceeds the sum
    assert mk['busy_ms'] <= wall_ms * 1.02 + 0.1     # nor the wall time around the calls
    assert mk['busy_ms'] >= 0.5 * wall_ms            # the megakernel is most of it
    # non-overlapped launches: busy == summed durations (disjoint intervals)
    with _lib.KernelTimer(max_launches=1000) as kt2:
        for k in range(3):
            integ.render_mk(fr, acc, 100 + k * spp, spp)
            torch.cuda.synchronize()
    mk2 = kt2.result['megakernel']
    assert abs(mk2['busy_ms'] - mk2['ms']) <= 1e-3 * max(1.0, mk2['ms'])


def test_mk_overlapped_batches_respect_the_item_id_limit():
    """render_mk(overlap=True) splits a call into batches that fit one
    ptmi_mk_trace_ws (ptmi_mk_max_batch), like the staged path above."""
    import ctypes as C
    import torch
    from edge_scenes import edge_scene
    from ptmi import device
    sa, cam, bg = edge_scene('empty')
    W, H = cam['width'], cam['height']
    integ = device.Integrator(device.DeviceScene.from_arrays(sa))
    fr = device.make_frame(cam, bg, 50, 0, W, H, (0, 0, 1, 1))
    mb = integ.lib.ptmi_mk_max_batch(C.byref(fr))
    assert mb == ((1 << 32) - 1) // (8 * 64)  # one tile, padded to the 8 unit shards
    n = 3 * mb + 5
    acc = torch.zeros((H, W, 3), dtype=torch.float32, device='cuda')
    integ.reset_counters()
    integ.render_mk(fr, acc, 0, n, overlap=True)
    torch.cuda.synchronize()
    assert integ.read_counters()['paths'] == n
    want = np.add.accumulate(np.full(n, np.float32(bg[0]), np.float32))[-1]
    assert acc[0, 0, 0].item() == want


def test_mk_overlapped_calls_on_changing_streams():
    """Overlapped calls whose caller stream changes from call to call, with a
    counter reset between calls and no synchronisation: the accumulator and
    the counters equal the plain same-stream calls bit for bit (each trace
    waits for the last resolve that read its workspace half and for the
    reset; each resolve for the previous resolve)."""
    import torch
    from ptmi import device
    sa, cam, bg = scene_inputs('vol2_final_scene', 800)
    integ = device.Integrator(device.DeviceScene.from_arrays(sa))
    fr = device.make_frame(cam, bg, 50, 0, cam['width'], cam['height'], (128, 256, 320, 192))
    calls = [(0, 5), (5, 3), (8, 6), (14, 2), (16, 4), (20, 3)]
    ref = torch.zeros((cam['height'], cam['width'], 3), dtype=torch.float32, device='cuda')
    for s0, n in calls[:2]:
        integ.render_mk(fr, ref, s0, n)
    integ.reset_counters()
    for s0, n in calls[2:]:
        integ.render_mk(fr, ref, s0, n)
    torch.cuda.synchronize()
    want_cnt = integ.read_counters()
    streams = [torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.current_stream()]
    acc = torch.zeros_like(ref)
    torch.cuda.synchronize()
    for j, (s0, n) in enumerate(calls):
        if j == 2:
            integ.reset_counters(stream=streams[j % 3])
        integ.render_mk(fr, acc, s0, n, stream=streams[j % 3], overlap=True)
    for s in streams:
        s.synchronize()
    torch.cuda.synchronize()
    assert torch.equal(acc, ref)
    assert integ.read_counters() == want_cnt


def test_multi_batch_overlapped_call_after_unsynchronised_reset():
    """A reset_counters(stream=...) with no synchronisation, followed by one
    overlapped call split into several batches: every batch's trace (each on
    its own side stream) runs after the reset, so the counters hold exactly
    that call's paths (only the first trace used to wait)."""
    import torch
    from ptmi import device
    sa, cam, bg = scene_inputs('vol2_final_scene', 800)
    integ = device.Integrator(device.DeviceScene.from_arrays(sa))
    fr = device.make_frame(cam, bg, 50, 0, cam['width'], cam['height'], (128, 256, 256, 128))
    npix = 256 * 128
    integ.STAGING_BYTES = 12 * npix * 2  # 2 samples per batch: a 6-sample call is 3 batches
    ref = torch.zeros((cam['height'], cam['width'], 3), dtype=torch.float32, device='cuda')
    integ.reset_counters()
    integ.render_mk(fr, ref, 10, 6)
    torch.cuda.synchronize()
    want = integ.read_counters()
    assert want['paths'] == 6 * npix
    acc = torch.zeros_like(ref)
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    for k in range(3):  # traces in flight on every side stream when the reset is queued
        integ.render_mk(fr, acc, 2 * k, 2, overlap=True)
    integ.reset_counters(stream=s)
    acc2 = torch.zeros_like(ref)
    integ.render_mk(fr, acc2, 10, 6, stream=s, overlap=True)
    s.synchronize()
    torch.cuda.synchronize()
    assert integ.read_counters() == want
    assert torch.equal(acc2, ref)


def test_profiler_with_concurrent_megakernel_threads():
    """ptmi_prof_* with render calls from several host threads: every launch
    gets its own event pair (no mixed-up begin/end), so the launch counts are
    exact and every duration is positive and bounded by the session."""
    import time
    import torch
    from ptmi import device, _lib
    sa, cam, _ = scene_inputs('vol2_final_scene', 800)
    dscene = device.DeviceScene.from_arrays(sa)
    n, calls = 3, 4
    integs = [device.Integrator(dscene) for _ in range(n)]
    accs = [_frame_acc(cam, (0, 0, 800, 800)) for _ in range(n)]
    streams = [torch.cuda.Stream() for _ in range(n)]
    for k in range(n):  # warm-up: workspaces
        integs[k].render_mk(accs[k][0], accs[k][1], 0, 2, stream=streams[k])
    torch.cuda.synchronize()
    errors = []
    start = threading.Barrier(n)

    def work(k):
        try:
            start.wait()
            for c in range(calls):
                integs[k].render_mk(accs[k][0], accs[k][1], 2 + 4 * c, 4, stream=streams[k])
            streams[k].synchronize()
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    with _lib.KernelTimer(max_launches=1000) as kt:
        t0 = time.perf_counter()
        threads = [threading.Thread(target=work, args=(k,)) for k in range(n)]
        for t in threads:
            t.start()
        for t in threads:
            t.join(timeout=120)
        torch.cuda.synchronize()
        wall_ms = (time.perf_counter() - t0) * 1e3
    assert not errors, errors
    mk, res = kt.result['megakernel'], kt.result['mk_resolve']
    assert mk['launches'] == n * calls == res['launches'] and not kt.truncated
    assert 0.0 < mk['busy_ms'] <= min(mk['ms'], wall_ms * 1.02 + 0.1)


def test_wavefront_tail_runs_in_one_drain_launch_per_pipe():
    """The wavefront's tail (wf_drain: once a pipe's live slots fall below
    capacity / 16 after the work pool ran dry, one launch finishes its paths)
    runs in every call that reaches it, and the render and the device counters
    still equal the oracle's (the drain runs the same per-path entry
    functions as wf_intersect / wf_scatter)."""
    import torch
    from parity_helpers import compare, oracle_render
    from ptmi import device, _lib
    sa, cam, bg = scene_inputs('vol2_final_scene', 800)
    integ = device.Integrator(device.DeviceScene.from_arrays(sa))
    win = (336, 352, 96, 64)
    fr = device.make_frame(cam, bg, 50, 0, cam['width'], cam['height'], win)
    acc = torch.zeros((cam['height'], cam['width'], 3), dtype=torch.float32, device='cuda')
    integ.reset_counters()
    with _lib.KernelTimer(max_launches=100000) as kt:
        integ.render_wf(fr, acc, 7, 8)
        torch.cuda.synchronize()
    drains = kt.result['wf_drain']['launches']
    assert 1 <= drains <= 4  # at most one per pipe and batch
    ref, ost = oracle_render('vol2_final_scene', 800, 'wf', win, 7, 8)
    linf, exact = compare(acc.cpu().numpy(), ref, 8)
    assert linf <= 1e-4 and exact >= 0.999
    assert integ.read_counters() == ost


_FULL_FRAME_ORACLE = {}


@pytest.mark.parametrize('drain_at', [1, 2, 0])
def test_wavefront_tail_traces_the_items_groups_still_hold(drain_at):
    """the tail launch starts once the work pool is dry
    and a pipe traces fewer than capacity / drain_at rays per iteration;
    wf_drain must then finish every path still in the pipe's ray buffer and
    lose none (no fresh item is due: the pool is dry). The whole 800x800
    frame x 8 spp is 5.12 M items for 2^22 rays per iteration, so the tail
    begins while the buffers are still well filled; drain_at = 1 starts it as
    soon as the pool is dry, 2 half-way, 0 never (one intersect + scatter
    launch per wave to the end). Every path is traced exactly once: the
    paths counter is W x H x spp, the image and the counters equal the
    oracle's bit for bit, and the tail traced segments whenever it ran."""
    import torch
    from parity_helpers import compare, oracle_render
    from ptmi import device, _lib
    sa, cam, bg = scene_inputs('vol2_final_scene', 800)
    W, H, spp = cam['width'], cam['height'], 8  # more items than the 2^22 rays per iteration
    lib = _lib.load()
    integ = device.Integrator(device.DeviceScene.from_arrays(sa))
    fr = device.make_frame(cam, bg, 50, 0, W, H)
    acc = torch.zeros((H, W, 3), dtype=torch.float32, device='cuda')
    integ.reset_counters()
    prev = lib.ptmi_wf_set_drain_at(drain_at)
    assert prev == 16
    try:
        with _lib.KernelTimer(max_launches=100000) as kt:
            integ.render_wf(fr, acc, 3, spp)
            torch.cuda.synchronize()
    finally:
        assert lib.ptmi_wf_set_drain_at(prev) == drain_at
    gst, tail = integ.read_counters(), integ.tail_segments()
    drains = kt.result['wf_drain']['launches']
    assert gst['paths'] == W * H * spp
    if drain_at:
        assert 1 <= drains <= 4 and 0 < tail <= gst['segments']
    else:
        assert drains == 0 and tail == 0
    if 'ref' not in _FULL_FRAME_ORACLE:
        _FULL_FRAME_ORACLE['ref'] = oracle_render('vol2_final_scene', 800, 'wf', (0, 0, W, H), 3, spp)
    ref, ost = _FULL_FRAME_ORACLE['ref']
    linf, exact = compare(acc.cpu().numpy(), ref, spp)
    assert linf == 0.0 and exact == 1.0
    assert gst == ost


def test_drain_divisor_is_validated():
    from ptmi import _lib
    lib = _lib.load()
    assert lib.ptmi_wf_set_drain_at(-1) == _lib.PTMI_EINVAL
    assert lib.ptmi_wf_set_drain_at(16) == 16


@pytest.mark.parametrize('win,band', [((400, 300, 1, 1), (1, 1, 0)), ((397, 301, 5, 3), (1, 1, 0)),
                                      ((390, 290, 21, 37), (4, 3, 1))])
def test_wavefront_multi_batch_and_ragged_windows(win, band):
    """The wavefront on ragged pixel sets — one pixel, a 5x3 window inside one
    8x8 square, a 21x37 window with every third 4-row band — and on a call
    split into several batches (a 2-sample staging budget: a 7-sample call is
    4 batches, each re-arming the pool, the segment counters and the status
    words): every path traced once, the image and the counters equal the
    oracle's bit for bit."""
    import torch
    from parity_helpers import compare, oracle_render
    from ptmi import device
    sa, cam, bg = scene_inputs('vol2_final_scene', 800)
    W, H = cam['width'], cam['height']
    integ = device.Integrator(device.DeviceScene.from_arrays(sa))
    fr = device.make_frame(cam, bg, 50, 0, W, H, win, band)
    rows = device.frame_pixel_rows(fr)
    npix = win[2] * len(rows)
    integ.STAGING_BYTES = 12 * npix * 2
    acc = torch.zeros((H, W, 3), dtype=torch.float32, device='cuda')
    integ.reset_counters()
    integ.render_wf(fr, acc, 5, 7)
    torch.cuda.synchronize()
    gst = integ.read_counters()
    assert gst['paths'] == npix * 7
    import oracle
    ofr = oracle.make_frame(cam, bg, 50, 0, W, H)
    ref = np.zeros((H, W, 3), np.float32)
    ost = {k: 0 for k in gst}
    osc = oracle.OracleScene(sa)
    for r in rows:  # the band's rows, one by one
        st = oracle.render(osc, ofr, 'wf', ref, (win[0], int(r), win[2], 1), 5, 7)
        for k in ost:
            ost[k] += st[k]
    linf, exact = compare(acc.cpu().numpy(), ref, 7)
    assert linf == 0.0 and exact == 1.0
    assert gst == ost
