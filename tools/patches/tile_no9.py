# A/B: without the 72-row (8 waves x 9 rows) tiles -- the dispatch rule before they were added
PATCHES = [
    ("(wg9 > 0 && ntiles9 <= cus) ||", "", 1),
    ("if (ntiles > cus && wg9 > 0 && ntiles9 <= cus) {", "if (false) {", 1),
]
