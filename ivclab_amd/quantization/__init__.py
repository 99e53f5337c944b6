from .patchquant import PatchQuant  # noqa: F401
