from . import net_ga, net_unet_ha_hs, source_net
from .gdn import GDN, IGDN
