from .reduce import reduce, reduce_host  # noqa: F401
