"""ORACLE (test infrastructure only): C restatement binding (filled in below)."""


def available() -> bool:
    return False
