"""Hand-built apply edge cases. Each case: table rows (kmer, role),
proteins, min_hits, flags. Expected outputs come from the Python twin (oracle/oracle_py.py)
and are frozen in tests/golden/apply_edge.json by tests/golden/gen_golden.py."""

F_END_EXCLUSIVE, F_MULTISET = 0x1, 0x2

A = "ACDEFGHI"      # 8-mers used as table kmers
B = "KLMNPQRS"
C = "TVWYACDE"
D = "MNPQRSTV"
E = "WYACDEFG"


def _chain(kmers):
    """A protein whose windows include every kmer of `kmers` (joined with one spacer)."""
    return "G".join(kmers)


CASES = [
    # name, rows, proteins, min_hits, flags
    ("short_protein", [(A, "R1")], ["", "A", "ACDEFGH"], 1, 0),
    ("exactly_k_inclusive", [(A, "R1")], [A], 1, 0),
    ("exactly_k_exclusive", [(A, "R1")], [A], 1, F_END_EXCLUSIVE),
    ("last_window_only", [(B, "R1")], ["AAAA" + B], 1, 0),
    ("last_window_exclusive", [(B, "R1")], ["AAAA" + B], 1, F_END_EXCLUSIVE),
    ("repeated_kmer_set", [(A, "R1"), (B, "R1")], [A + A + B + A], 1, 0),
    ("repeated_kmer_multiset", [(A, "R1"), (B, "R1")], [A + A + B + A], 1, F_MULTISET),
    ("ambiguous_two_roles", [(A, "R1"), (B, "R2")], [_chain([A, B])], 1, 0),
    ("ambiguous_many", [(A, "R1"), (B, "R1"), (C, "R1"), (D, "R2")],
     [_chain([A, B, C, D]), _chain([D, A, B, C])], 1, 0),
    ("min_hits_boundary", [(A, "R1"), (B, "R1"), (C, "R1"), (D, "R1"), (E, "R1")],
     [_chain([A, B, C, D]), _chain([A, B, C, D, E])], 5, 0),
    ("duplicate_db_key_last_wins", [(A, "R1"), (B, "R2"), (A, "R2")], [_chain([A, B])], 1, 0),
    ("duplicate_db_key_last_wins_2", [(A, "R2"), (A, "R1"), (B, "R2")], [_chain([A, B])], 1, 0),
    ("db_kmer_wrong_length", [("ACDEFGH", "R1"), ("ACDEFGHIK", "R1"), (B, "R2")],
     [A + "K", B], 1, 0),
    ("x_and_stop_are_plain_residues", [("ACDXFGHI", "R1"), ("KLMNPQR*", "R1")],
     ["ACDXFGHIKLMNPQR*"], 1, 0),
    ("lowercase_does_not_match", [(A, "R1")], [A.lower(), A], 1, 0),
    ("foreign_symbols", [("ACDE-GHI", "R1"), ("AC.EFGHI", "R1"), ("ACDEFGH1", "R2")],
     ["ACDE-GHI", "xAC.EFGHI", "ACDEFGH1", "ACDE#GHI"], 1, 0),
    ("role_order_first_seen", [(B, "R9"), (A, "R3"), (C, "R9")], [_chain([A]), _chain([B, C])],
     1, 0),
    ("no_hits", [(A, "R1")], ["KKKKKKKKKKKKKKKK", "WWWWWWWWW"], 1, 0),
]
