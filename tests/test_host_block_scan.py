"""CPU-side half of the no-host-sync check (verdict r03 item 8): every host-blocking HIP runtime
call in the engine's sources goes through ZV_BLOCKING (zv_common.h), which counts it, so the GPU
test (tests/test_gpu_host_sync.py) that asserts a zero count across a warm step sees every such
call.  A source scan: blocking calls written without the wrapper fail here."""
import pathlib
import re

CSRC = pathlib.Path(__file__).resolve().parents[1] / "zipvoice_amd" / "csrc"
BLOCKING = ["hipMalloc", "hipMallocManaged", "hipHostMalloc", "hipMemcpy", "hipMemcpy2D", "hipFree",
            "hipHostFree", "hipMemset", "hipDeviceSynchronize", "hipEventSynchronize",
            "hipStreamSynchronize", "hipGraphInstantiate", "hipStreamCreate",
            "hipStreamCreateWithFlags", "hipStreamCreateWithPriority", "hipEventCreate",
            "hipEventCreateWithFlags", "hipStreamDestroy", "hipEventDestroy", "hipGraphDestroy",
            "hipGraphExecDestroy", "hipEventQuery", "hipStreamQuery"]


def _calls(text):
    pat = re.compile(r"\b(%s|hipMemcpyAsync)\(" % "|".join(BLOCKING))
    for m in pat.finditer(text):
        line_start = text.rfind("\n", 0, m.start()) + 1
        if text[line_start:m.start()].lstrip().startswith("//"):
            continue
        depth, j = 0, m.end() - 1
        while True:
            depth += {"(": 1, ")": -1}.get(text[j], 0)
            if depth == 0:
                break
            j += 1
        yield m.group(1), m.start(), text[m.start():j + 1], text.count("\n", 0, m.start()) + 1


def test_blocking_calls_are_counted():
    files = sorted(CSRC.glob("*.hip")) + sorted(CSRC.glob("*.inc")) + sorted(CSRC.glob("*.h"))
    assert files
    seen, bad = 0, []
    for f in files:
        text = f.read_text()
        for name, pos, call, line in _calls(text):
            if name == "hipMemcpyAsync" and "DeviceToHost" not in call:
                continue                      # device-side copies are queued, not blocking
            seen += 1
            if not text[:pos].endswith("ZV_BLOCKING("):
                bad.append(f"{f.name}:{line}: {call[:80]}")
    assert seen > 50                          # the scan really sees the engine's runtime calls
    assert not bad, "host-blocking calls outside ZV_BLOCKING:\n" + "\n".join(bad)


def test_counter_exported():
    """The counter is part of the C ABI (declared in include/zipvoice_hip.h, bound in engine.py)."""
    from zipvoice_amd.engine import SIGNATURES
    hdr = (CSRC.parents[1] / "include" / "zipvoice_hip.h").read_text()
    assert "int64_t zv_host_block_count(void);" in hdr
    assert "zv_host_block_count" in SIGNATURES
