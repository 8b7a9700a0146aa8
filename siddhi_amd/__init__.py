"""siddhi_amd — MI355X (gfx950) execution path for Siddhi pattern / sequence matching over
windowed streams, behind the reference's SiddhiManager / InputHandler / callback API.

The compute path is libsiddhi_gfx.so (HIP kernels + C ABI, include/siddhi_gfx.h); this package
holds the QL front-end that emits the descriptor and the Python mirror of the public API.
"""
from .ql import compile_app, parse_app, SiddhiParserError  # noqa: F401
from .runtime import (Event, GpuApp, InputHandler, QueryCallback, SiddhiAppRuntime,  # noqa: F401
                      SiddhiGfxError, SiddhiManager, StreamCallback, lib)
