"""tools/trace_intervals.py: the union of kernel dispatch intervals that checks bench.py's kernel_ms against a
rocprofv3 kernel trace (pipelined sample launches).  CPU only: synthetic trace rows."""
import importlib.util
import pathlib

import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
spec = importlib.util.spec_from_file_location("trace_intervals", ROOT / "tools" / "trace_intervals.py")
TI = importlib.util.module_from_spec(spec)
spec.loader.exec_module(TI)


def rows(*iv):
    return [{"Start_Timestamp": str(int(a * 1e6)), "End_Timestamp": str(int(b * 1e6))} for a, b in iv]


def test_series_adds_durations():
    assert TI.throughput_ms(rows((0, 10), (12, 22), (22, 30))) == pytest.approx([10, 10, 8])


def test_overlapped_launches_count_from_the_previous_end():
    # dispatched while the previous launch drains: each counts from the previous end
    assert TI.throughput_ms(rows((0, 146), (140, 292), (285, 438))) == pytest.approx([146, 146, 146])


def test_side_by_side_and_out_of_order_launches_count_once():
    # two slots' launches dispatched together, the later one run first (as the r05b trace showed):
    # the union is the busy time, whatever the order in which they end
    got = TI.throughput_ms(rows((353.38, 499.30), (353.65, 644.82), (499.54, 790.37)))
    assert sum(got) == pytest.approx(790.37 - 353.38)
    assert all(x >= 0 for x in got)
    # a launch wholly inside another's interval adds nothing
    assert TI.throughput_ms(rows((0, 100), (10, 50))) == pytest.approx([100, 0])
