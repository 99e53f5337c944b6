"""Module `__getattr__` for the reference names this package leaves out on purpose.

A listed name raises `OutOfScopeError` (an ImportError) whose message says why: the name is
outside the MI355X block-codec hot path.  It is deliberately NOT an
AttributeError: `from ivclab.signal import downsample` turns an AttributeError from a module
`__getattr__` into a bare "cannot import name" ImportError, which would drop the reason; an
ImportError passes through unchanged, on the from-import and on plain attribute access alike.
Names that are not listed raise the usual AttributeError."""


class OutOfScopeError(ImportError):
    """A reference name outside the hot path this package implements."""


def out_of_scope(module_name, names):
    names = dict(names)

    def __getattr__(attr):
        if attr in names:
            raise OutOfScopeError(
                f"{module_name}.{attr} ({names[attr]}) is outside the MI355X block-codec "
                f"hot path this package implements (DESIGN.md §8)", name=attr)
        raise AttributeError(f"module {module_name!r} has no attribute {attr!r}")
    return __getattr__
