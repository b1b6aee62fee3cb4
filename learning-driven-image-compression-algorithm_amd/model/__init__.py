from . import net_ga, net_unet_ha_hs
from .gdn import GDN, IGDN
