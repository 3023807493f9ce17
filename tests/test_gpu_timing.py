"""Kernel time of the sample launches (srt_last_kernel_ms / srt_kernel_time): each launch's own span on
the GPU clock, as bench.py reads it once after a timed loop of renders enqueued back to back."""
import pytest

import srt_amd as S
from srt_amd import render as R
from conftest import OBJECTS

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("scene", ["rubik", "spheres"])
def test_kernel_time_counts_every_launch(scene):
    setup = (R.make_setup(320, 192, show_model=False, max_depth=4) if scene == "spheres"
             else R.make_setup(320, 192, show_model=True, models=[S.load_obj(OBJECTS / "Rubik" / "Rubik.obj")]))
    r = R.Renderer(setup)
    try:
        r.render(16, count=True)
        r.finish()
        r.compute.kernel_time()  # drops the counting launch
        for _ in range(4):  # back to back, no finish between them
            r.render(16)
        last = r.compute.last_kernel_ms()
        total, launches = r.compute.kernel_time()
        assert launches == 4
        assert last > 0.0 and total > 0.0
        # every launch renders the same frames: the sum is about four times the last one
        assert 2.0 * last < total < 8.0 * last
        assert r.compute.kernel_time() == (0.0, 0)  # nothing launched since
    finally:
        r.close()
