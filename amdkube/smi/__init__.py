from .backend import (Backend, AmdSmiBackend, SysfsBackend, FakeBackend, open_backend, device_id, visibility_token,  # noqa: F401
                      SMIError, DEFAULT_FIXTURE)
