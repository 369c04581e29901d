"""The ``useGpu`` query option routes between the GPU operators and the CPU plan maker
(InstancePlanMakerImplV2.makeInstancePlan override). Host-only: no segment is touched."""
import pytest

from pinot_amd.engine.plan import GpuInstancePlanMaker, UnsupportedOnGpu, use_gpu_option
from pinot_amd.query.sql import parse


class _CpuMaker:
    def __init__(self):
        self.calls = []

    def make_instance_plan(self, query, segments):
        self.calls.append(query)
        return ("cpu-plan", query)


def test_option_parsing_follows_boolean_parse_boolean():
    assert use_gpu_option(parse("SET useGpu = true; SELECT COUNT(*) FROM t"), False)
    assert use_gpu_option(parse("SET useGpu = 'TRUE'; SELECT COUNT(*) FROM t"), False)
    assert not use_gpu_option(parse("SET useGpu = false; SELECT COUNT(*) FROM t"), True)
    assert not use_gpu_option(parse("SET useGpu = yes; SELECT COUNT(*) FROM t"), True)  # parseBoolean("yes") = false
    assert use_gpu_option(parse("SELECT COUNT(*) FROM t"), True)
    assert not use_gpu_option(parse("SELECT COUNT(*) FROM t"), False)


def test_use_gpu_false_goes_to_the_cpu_plan_maker():
    cpu = _CpuMaker()
    q = parse("SET useGpu = false; SELECT COUNT(*) FROM t")
    plan = GpuInstancePlanMaker(cpu_plan_maker=cpu).make_instance_plan(q, [])
    assert plan[0] == "cpu-plan" and cpu.calls == [q]


def test_use_gpu_false_without_a_cpu_plan_maker_raises():
    with pytest.raises(UnsupportedOnGpu):
        GpuInstancePlanMaker().make_instance_plan("SET useGpu = false; SELECT COUNT(*) FROM t", [])


def test_server_default_off_routes_queries_without_the_option_to_cpu():
    cpu = _CpuMaker()
    pm = GpuInstancePlanMaker(cpu_plan_maker=cpu, default_use_gpu=False)
    assert pm.make_instance_plan("SELECT COUNT(*) FROM t", [])[0] == "cpu-plan"


def test_query_outside_the_gpu_subset_falls_back():
    cpu = _CpuMaker()
    q = "SET useGpu = true; SELECT SUM(a / b) FROM t"
    assert GpuInstancePlanMaker(cpu_plan_maker=cpu).make_instance_plan(q, [])[0] == "cpu-plan"
    with pytest.raises(UnsupportedOnGpu):
        GpuInstancePlanMaker().make_instance_plan(q, [])
