"""Timing-only ablation (no outputs): the row stream's back issues no global stores (st_nt is empty)."""
PATCHES = [
    ('    asm volatile("global_store_dwordx4 %0, %1, off nt\\n\\ts_nop 1" :: "v"(p), "v"(x) : "memory");',
     '    asm volatile("" :: "v"(p), "v"(x) : "memory");', 1),
]
