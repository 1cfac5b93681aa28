"""Helpers mirrored from the reference's decentralizepy/utils.py (used by the plugin kwargs)."""


def conditional_value(var, nul, default):
    """reference utils.py:7-29: ``default`` if ``var == nul`` else ``var``."""
    if var != nul:
        return var
    return default


def identity(obj):
    """reference utils.py:126-138 (PartialModel's default change_transformer)."""
    return obj
