"""DeviceShare with reservations that hold devices (deviceshare/reservation.go) on the C oracle, pinned by the
reference's own tests (tests/golden/deviceshare_reservation.json, transcribed from deviceshare/reservation_test.go):
RestoreReservation's merged restore state (Test_Plugin_ReservationRestore) and tryAllocateFromReservation over the
Default / Aligned / Restricted policies (Test_tryAllocateFromReservation), through test hooks of the oracle."""
import ctypes as C
import json
import pathlib

import numpy as np
import pytest

from koordinator_amd import abi, synth
from koordinator_amd.cluster import DeviceTable, NodeTable, PodTable, ReservationTable
from koordinator_amd.config import DeviceShareArgs
from oracle.oracle import Oracle

G = json.loads((pathlib.Path(__file__).parent / "golden" / "deviceshare_reservation.json").read_text())
GIB = G["gib"]
POLICY = {"Default": abi.KS_RSV_POLICY_DEFAULT, "Aligned": abi.KS_RSV_POLICY_ALIGNED,
          "Restricted": abi.KS_RSV_POLICY_RESTRICTED}


def words(minors: dict) -> np.ndarray:
    w = np.zeros(abi.KS_DEV_WORDS, np.int64)
    for k, (core, mem, ratio) in minors.items():
        k = int(k)
        w[abi.dev_word("gpu", k, 0)] = core
        w[abi.dev_word("gpu", k, 1)] = mem * GIB
        w[abi.dev_word("gpu", k, 2)] = ratio
    return w


def cluster(gpus: dict, used: dict, rows: list):
    nodes = NodeTable(1)
    nodes.alloc_milli_cpu[:] = 64000
    nodes.alloc_memory[:] = 256 * GIB
    nodes.allowed_pods[:] = 110
    dev = DeviceTable(1)
    dev.flags[:] = abi.KS_DEV_PRESENT
    for k, (core, mem, ratio) in gpus.items():
        dev.total_core[int(k), 0], dev.total_memory[int(k), 0], dev.total_ratio[int(k), 0] = core, mem * GIB, ratio
    for k, (core, mem, ratio) in used.items():
        dev.used_core[int(k), 0], dev.used_memory[int(k), 0], dev.used_ratio[int(k), 0] = core, mem * GIB, ratio
    rs = ReservationTable(len(rows)).hold_devices()
    for i, (pol, al, ald, assigned) in enumerate(rows):
        rs.owner_classes[i] = 1
        rs.policy[i] = pol
        rs.key_mask[i] = 0b11
        rs.allocatable[0, i] = 1000
        rs.assigned[i] = assigned
        rs.dev_allocatable[i] = al
        rs.dev_allocated[i] = ald
    prof = synth.koord_profile(with_reservation=True)
    prof.deviceshare = DeviceShareArgs()
    return Oracle(prof.to_ks_config(), nodes, reservations=rs, devices=dev)


def gpu_pod(core: int, mem_or_ratio: int, by_memory: bool) -> PodTable:
    p = PodTable(1)
    p.req_milli_cpu[:] = 100
    p.nonzero_milli_cpu[:] = 100
    p.nonzero_memory[:] = 200 << 20
    p.rsv_class[:] = 0
    p.gpu_core[:] = core
    if by_memory:
        p.gpu_memory[:] = mem_or_ratio * GIB
        p.flags[:] = abi.KS_POD_GPU_CORE | abi.KS_POD_GPU_MEMORY
    else:
        p.gpu_memory_ratio[:] = mem_or_ratio
        p.flags[:] = abi.KS_POD_GPU_CORE
    return p


def test_reservation_restore_state():
    c = G["restore"]
    r = c["reservation"]
    orc = cluster(c["gpus"], c["used"], [(abi.KS_RSV_POLICY_DEFAULT, words(r["allocatable"]), words(r["allocated"]),
                                          r["assigned"])])
    pod = gpu_pod(c["pod"]["core"], c["pod"]["ratio"], False)
    pc = pod.ks()
    uu, mm, am = (np.zeros(abi.KS_DEV_WORDS, np.int64) for _ in range(3))
    orc.L.ko_test_device_restore.argtypes = [C.c_void_p, C.POINTER(abi.KsPodCols), C.c_int64, abi.P64, abi.P64, abi.P64]
    nm = orc.L.ko_test_device_restore(orc.h, C.byref(pc), 0, *(a.ctypes.data_as(abi.P64) for a in (uu, mm, am)))
    w = c["want"]
    assert nm == w["matched"]
    assert np.array_equal(uu, words(w["merged_unmatched_used"]))
    assert np.array_equal(am, words(w["merged_matched_allocatable"]))
    assert np.array_equal(mm, words(w["merged_matched_allocated"]))
    orc.close()


@pytest.mark.parametrize("case", G["try_allocate"]["cases"], ids=lambda c: c["name"][:60])
def test_try_allocate_from_reservation(case):
    rows = [(POLICY[m["policy"]], words(m["allocatable"]), words(m["allocatable"]) - words(m["remained"]), 1)
            for m in case["matched"]]
    orc = cluster(G["try_allocate"]["gpus"], case["used"], rows or [(0, np.zeros(abi.KS_DEV_WORDS, np.int64),
                                                                     np.zeros(abi.KS_DEV_WORDS, np.int64), 0)])
    pod = gpu_pod(case["pod"][0], case["pod"][1], True)
    pc = pod.ks()
    idx = np.arange(len(case["matched"]), dtype=np.int32)
    uu = np.zeros(abi.KS_DEV_WORDS, np.int64)
    mm = words(case["mm"])
    out = np.zeros(2, np.uint32)
    L = orc.L
    L.ko_test_try_reservation.argtypes = [C.c_void_p, C.POINTER(abi.KsPodCols), C.c_int64, abi.P32, C.c_int32, abi.P64,
                                          abi.P64, C.c_int32, abi.PU32]
    rc = L.ko_test_try_reservation(orc.h, C.byref(pc), 0, idx.ctypes.data_as(abi.P32), len(idx),
                                   uu.ctypes.data_as(abi.P64), mm.ctypes.data_as(abi.P64), int(case["required"]),
                                   out.ctypes.data_as(abi.PU32))
    want = case["want"]
    if want is None:
        assert rc == 0
    elif want == "unschedulable":
        assert rc == -1
    else:
        assert rc == 1 and out[0] == sum(1 << k for k in want) and out[1] == 0
    orc.close()
