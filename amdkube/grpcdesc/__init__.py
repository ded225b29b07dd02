from .compiler import ProtoModule, Service  # noqa: F401
