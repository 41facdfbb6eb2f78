"""Console banner + network summary (reference tensordiffeq/output.py:5-11, which used pyfiglet
and the Keras ``model.summary()``; pyfiglet is not a dependency here, the banner is built in)."""
from __future__ import annotations

_BANNER = r"""
  _____                         ____  _  __  __ _____
 |_   _|__ _ __  ___  ___  _ __|  _ \(_)/ _|/ _| ____|__ _
   | |/ _ \ '_ \/ __|/ _ \| '__| | | | | |_| |_|  _| / _` |
   | |  __/ | | \__ \ (_) | |  | |_| | |  _|  _| |__| (_| |
   |_|\___|_| |_|___/\___/|_|  |____/|_|_| |_| |_____\__, |
                          MI355X / HIP edition           |_|
"""


def banner():
    return _BANNER


def print_screen(model, discovery_model=False):
    print(_BANNER)
    if discovery_model:
        print("Running Discovery Model for Parameter Estimation\n\n")
    print("Neural Network Model Summary\n")
    net = getattr(model, "u_model", None)
    summary = getattr(net, "summary", None)
    print(summary() if callable(summary) else repr(net))
    prog = None
    try:
        prog = model.program()
    except Exception:  # pragma: no cover - summary must never break training
        pass
    if prog is not None:
        print(f"\nbackend: {prog.backend}" + (f"  streams: {prog.plan.streams}" if prog.plan else ""))
