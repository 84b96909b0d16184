from .amp_utils import get_autocast, get_input_dtype  # noqa: F401
from .dist_utils import (broadcast_object, init_device, is_global_master, is_local_master, is_master,  # noqa: F401
                         is_using_distributed, world_info_from_env)
