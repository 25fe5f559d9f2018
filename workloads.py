"""The BASELINE.json config workloads as request lists, shared by bench_configs.py
(timing) and tests/test_configs_gpu.py (oracle parity at the same geometry).

  C4  SmartCrop 256x256 (reference image.go:236-245), Thumbnail 256x256
      (:279-284) + WatermarkImage 128x128 RGBA at (16, 16), opacity 0.5
      (:343-370), on 12 MP decoded inputs 4000x3000 and 3000x4000 RGB
  C5  mixed request stream over {1080p, 4K, 12 MP} RGB, seed 5:
      40 % resize width {300, 640, 1280}, 20 % fit 800x800, 15 % rotate,
      15 % embed to 1:1 with a random extend, 10 % blur sigma {1, 3, 5}
"""
import numpy as np

C4_SIZES = ((4000, 3000), (3000, 4000))
C4_WM_SHAPE = (128, 128, 4)  # (h, w, bands)
C4_OPTS = (
    dict(width=256, height=256, crop=1, gravity=5),                                   # SmartCrop
    dict(width=256, height=256, wm_enable=1, wm_left=16, wm_top=16, wm_opacity=0.5),  # Thumbnail + watermark
)


def c4_watermark(seed=4):
    return np.random.default_rng(seed).integers(0, 256, C4_WM_SHAPE, dtype=np.uint8)


def c5_requests(count, seed=5, fit_dimension=None):
    """[((w, h), opts)] for `count` requests; fit_dimension(iw, ih, fw, fh) is the
    engine's mipx_fit_dimension (imaginary image.go:190)."""
    if fit_dimension is None:
        import imaginary_amd as ia
        fit_dimension = ia.fit_dimension
    r = np.random.default_rng(seed)
    sizes = [(1920, 1080), (3840, 2160), (4000, 3000)]
    reqs = []
    for _ in range(count):
        w, h = sizes[r.integers(0, 3)]
        u = r.random()
        if u < 0.40:
            opts = dict(width=int(r.choice([300, 640, 1280])), embed=1)
        elif u < 0.60:
            fw, fh = fit_dimension(w, h, 800, 800)
            opts = dict(width=fw, height=fh, embed=1)
        elif u < 0.75:
            opts = dict(rotate=int(r.choice([90, 180, 270])))
        elif u < 0.90:
            s = max(w, h)
            opts = dict(width=s, height=s, embed=1, extend=int(r.choice([0, 1, 2, 3, 4, 5])))
        else:
            opts = dict(sigma=float(r.choice([1.0, 3.0, 5.0])))
        reqs.append(((w, h), opts))
    return reqs


def c5_groups(reqs):
    """Requests grouped by identical plan input: [((w, h), opts, count)], sorted."""
    import json
    buckets = {}
    for (w, h), opts in reqs:
        key = (w, h, json.dumps(opts, sort_keys=True))
        buckets.setdefault(key, [0, opts])[0] += 1
    return [((w, h), opts, cnt) for (w, h, _), (cnt, opts) in sorted(buckets.items())]


def shard_groups(groups, world, bytes_per_request):
    """Split the plan groups [((w, h), opts, count)] over `world` ranks by bytes
    (greedy, largest first), keeping each group on as few ranks as
    possible: a group goes whole to the least-loaded rank while it fits under the
    per-rank target, and only the part that does not fit spills to the next
    least-loaded rank.  bytes_per_request((w, h), opts) is the request's input +
    output bytes.  Returns one group list per rank, same form as the input."""
    sized = [((w, h), opts, cnt, bytes_per_request((w, h), opts)) for (w, h), opts, cnt in groups]
    total = sum(cnt * b for _, _, cnt, b in sized)
    target = total / world
    load = [0] * world
    out = [[] for _ in range(world)]
    for (w, h), opts, cnt, b in sorted(sized, key=lambda g: (-g[2] * g[3], g[0], str(sorted(g[1].items())))):
        left = cnt
        while left > 0:
            r = min(range(world), key=lambda k: (load[k], k))
            room = -int(-(target - load[r]) // b) if b else left  # ceil: a rank fills to the target once
            take = left if room >= left else max(1, room)
            out[r].append(((w, h), opts, take))
            load[r] += take * b
            left -= take
    return out
