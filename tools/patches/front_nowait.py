"""Timing-only variant (wrong data): the stream kernel's front does not wait for its row's LDS-DMA loads before the
data term -- whether the loads issued 4 steps ahead still expose HBM latency to the step."""
PATCHES = [
    ("wait_vm<4>();   // row q's loads landed; parts 0-2 of row q + 4 may fly", "", 1),
]
