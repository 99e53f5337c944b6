"""Module `__getattr__` for the reference names this package leaves out on purpose.

`from ivclab.signal import downsample` then fails with an ImportError whose message
says why (the name is outside the MI355X block-codec hot path), rather
than a bare "cannot import name"."""


def out_of_scope(module_name, names):
    names = dict(names)

    def __getattr__(attr):
        if attr in names:
            raise AttributeError(
                f"{module_name}.{attr} ({names[attr]}) is outside the MI355X block-codec "
                f"hot path this package implements (DESIGN.md §8)")
        raise AttributeError(f"module {module_name!r} has no attribute {attr!r}")
    return __getattr__
