"""The Strings behind the HANDLE keys of the synthetic map streams (copycat_amd/csrc/workload.cpp draws handle keys
below `keys`): handle h is the String f"key-{h}".  java.util.HashMap places a String key by String.hashCode, so the
engine (cc_handle_hashes) and the oracle (orc_handle_string) both need them for MapState's iteration order."""


def key_strings(n=8192):
    return {h: f"key-{h}" for h in range(n)}


def register_key_strings(E=None, O=None, n=8192):
    s = key_strings(n)
    if E is not None:
        E.handle_strings(s)
    if O is not None:
        for h, x in s.items():
            O.handle_string(h, x)
