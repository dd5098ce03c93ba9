from openfl_amd.workloads import WORKLOADS, numel


def test_workload_sizes():
    want = {"mnist_cnn": (8, 431_080), "resnet50_fp32": (267, 25_610_152),
            "uniform_1gib": (64, 2 ** 28), "llama3_8b_fp32_update": (291, 8_030_261_248)}
    for name, (count, total) in want.items():
        shapes = WORKLOADS[name]()
        assert len(shapes) == count
        assert sum(numel(s) for _, s in shapes) == total
