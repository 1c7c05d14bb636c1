"""The ctypes stub INTEGRATION.md §3 gives a reference maintainer must
declare the ABI structs with the sizes the library's own binding
(gamesmanmpi_amd/_lib.py) uses: a short struct would let gm_solver_solve
write past the caller's memory."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_integration_stub_struct_sizes_match_the_binding():
    from gamesmanmpi_amd import _lib
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    code = re.search(r"```python\n(.*?)```", text, re.S).group(1)
    stub = code.split("gid = ctypes.c_int()")[0]  # the struct declarations only
    ns = {}
    exec(stub.replace('lib = ctypes.CDLL("gamesmanmpi_amd/libgamesman_hip.so")', "")
         .replace("import ctypes, torch", "import ctypes"), ns)
    assert ctypes.sizeof(ns["Plan"]) == ctypes.sizeof(_lib.gm_plan_t)
    assert ctypes.sizeof(ns["Buffers"]) == ctypes.sizeof(_lib.gm_buffers)
    assert ctypes.sizeof(ns["Result"]) == ctypes.sizeof(_lib.gm_result)


def test_binding_structs_match_the_compiled_abi():
    """_lib's ctypes structs against sizeof() inside the library."""
    import numpy as np
    from gamesmanmpi_amd import _lib
    out = np.zeros(3, np.uint32)
    _lib.check(_lib.load().gm_abi_sizes(out.ctypes.data))
    assert out.tolist() == [ctypes.sizeof(_lib.gm_plan_t), ctypes.sizeof(_lib.gm_buffers),
                            ctypes.sizeof(_lib.gm_result)]
