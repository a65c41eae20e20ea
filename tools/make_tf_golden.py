"""Golden TF texels for SURVEY.md §8 row f2 (the TF producer), from an independent float32
restatement of the reference's published formulas -- not from the product code:

  * Gradient() markers: colour (0, black), (1, white); alpha (0, 1), (1, 1)
    (/root/reference/src/ui/components/gradient.cpp:64-70);
  * discretize(count): stride = 1/count, location starts at stride/2 and is ACCUMULATED in
    float (location += stride), one texel per step (gradient.cpp:90-108);
  * sample_markers: clamp to [0, 1], lower_bound on marker.location < location, first/last
    marker values outside, else lerp(a, b, t) = a * (1 - t) + b * t with
    t = (location - prev) / (curr - prev) (gradient.cpp:13-16, 471-485);
  * ImGui::ColorConvertFloat4ToU32: IM_F32_TO_INT8_SAT(v) = (int)(saturate(v) * 255.0f + 0.5f),
    R | G << 8 | B << 16 | A << 24 (imgui, unversioned submodule: the published macro).

Every operation is float32 (numpy scalars), no fused multiply-add, as an x86-64 build of the
reference computes them.  Writes tests/golden/tf_golden.json; tests/test_host.py checks the
product's vr_gradient_* against it exactly and re-runs this script to check the fixture.
Usage: python tools/make_tf_golden.py [out.json]
"""
import json
import os
import sys

import numpy as np

F = np.float32


def sample_markers(markers, location):
    location = min(max(location, F(0.0)), F(1.0))
    i = 0
    while i < len(markers) and markers[i][0] < location:  # std::lower_bound
        i += 1
    if i == 0:
        return markers[0][1]
    if i == len(markers):
        return markers[-1][1]
    curr, prev = markers[i][0], markers[i - 1][0]
    t = F(F(location - prev) / F(curr - prev))
    a, b = markers[i - 1][1], markers[i][1]
    one_t = F(F(1.0) - t)
    return tuple(F(F(x * one_t) + F(y * t)) for x, y in zip(a, b))


def to_u8(v):
    s = min(max(v, F(0.0)), F(1.0))
    return int(F(F(s * F(255.0)) + F(0.5)))


def discretize(color, alpha, count=256):
    stride = F(F(1.0) / F(count))
    location = F(stride / F(2.0))
    out = []
    for _ in range(count):
        c = sample_markers(color, location)
        a = sample_markers(alpha, location)[0]
        out.append(to_u8(c[0]) | to_u8(c[1]) << 8 | to_u8(c[2]) << 16 | to_u8(a) << 24)
        location = F(location + stride)
    return out


def markers(pairs):
    return [(F(loc), tuple(F(x) for x in (v if isinstance(v, (tuple, list)) else (v,)))) for loc, v in pairs]


TFS = {
    # TF-1: the default Gradient() (gradient.cpp:64-70), discretize(256) (main_window.cpp:252)
    "tf1": dict(color=[(0.0, (0.0, 0.0, 0.0)), (1.0, (1.0, 1.0, 1.0))],
                alpha=[(0.0, 1.0), (1.0, 1.0)]),
    # TF-2: the demo-GIF ramp: colour black -> white, alpha markers (0, 0), (0.14, 0), (1, 1)
    "tf2": dict(color=[(0.0, (0.0, 0.0, 0.0)), (1.0, (1.0, 1.0, 1.0))],
                alpha=[(0.0, 0.0), (0.14, 0.0), (1.0, 1.0)]),
    # a coloured TF with three colour markers and partial alpha (tools/synth.py tf_color)
    "tf_color": dict(color=[(0.0, (0.1, 0.2, 0.9)), (0.5, (0.9, 0.1, 0.1)), (1.0, (1.0, 0.9, 0.2))],
                     alpha=[(0.0, 0.02), (1.0, 0.35)]),
}


def build():
    res = {}
    for name, m in TFS.items():
        for count in (256, 7):
            res[f"{name}_{count}"] = dict(color_markers=m["color"], alpha_markers=m["alpha"],
                                          count=count,
                                          texels=discretize(markers(m["color"]), markers(m["alpha"]), count))
    return res


if __name__ == "__main__":
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "tf_golden.json")
    json.dump(build(), open(out, "w"))
    print("wrote", out)
