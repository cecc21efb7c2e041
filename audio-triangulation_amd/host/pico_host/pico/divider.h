/* Host platform layer: no hardware divider on the host. */
#pragma once
