"""Module `__getattr__` for the reference names this package leaves out on purpose.

A listed name raises an error whose message says why: the name is outside the MI355X
block-codec hot path.  Which error depends on how the name was asked for:

* `from ivclab.signal import downsample` raises `OutOfScopeError` (an ImportError).  An
  AttributeError from a module `__getattr__` would be turned into a bare "cannot import name"
  ImportError by the interpreter, which drops the reason.
* attribute access (`ivclab.signal.downsample`, `hasattr`, `getattr(m, name, default)`, mocks,
  feature probes) raises `OutOfScopeAttributeError` (an AttributeError), so `hasattr` returns
  False and `getattr` with a default returns the default, as on the reference's modules when a
  name is absent.

The two cannot be one class: ImportError and AttributeError have conflicting instance layouts.
The from-import is recognised by the opcode the calling frame is executing (IMPORT_FROM).
Names that are not listed raise the usual AttributeError."""
import dis
import sys

_IMPORT_FROM = dis.opmap["IMPORT_FROM"]


class OutOfScopeError(ImportError):
    """A reference name outside the hot path this package implements (from-import form)."""


class OutOfScopeAttributeError(AttributeError):
    """The same, on attribute access: hasattr() is False, getattr(..., default) returns it."""


def _in_from_import(depth: int = 2) -> bool:
    try:
        f = sys._getframe(depth)
    except ValueError:
        return False
    i = f.f_lasti
    code = f.f_code.co_code
    return 0 <= i < len(code) and code[i] == _IMPORT_FROM


def out_of_scope(module_name, names):
    names = dict(names)

    def __getattr__(attr):
        if attr in names:
            msg = (f"{module_name}.{attr} ({names[attr]}) is outside the MI355X block-codec "
                   f"hot path this package implements (DESIGN.md §8)")
            if _in_from_import():
                raise OutOfScopeError(msg, name=attr)
            raise OutOfScopeAttributeError(msg)
        raise AttributeError(f"module {module_name!r} has no attribute {attr!r}")
    return __getattr__
