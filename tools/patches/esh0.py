"""Timing-only variant (wrong noise for W % 4 != 0): every row's noise quads taken as row-aligned, so the
second-quad path never runs -- measures what row-aligned noise quads would save in the stream and tile kernels."""
PATCHES = [
    ("esh = (int)(e & 3);                         // the same for every lane of the row", "esh = 0;", 1),
    ("const int esh = (int)(e & 3);               // the same for every lane of the row", "const int esh = 0;", 1),
]
