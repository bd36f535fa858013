"""Mirror of the reference module ax.xz.wireguard.noise (crypto + handshake
packages) whose ChaCha20-Poly1305 arithmetic runs on the MI355X through
libwgaead. Same class and method names, argument meaning and exceptions as the
Java sources, so the reference's own tests read the same against it."""
from .crypto import (AEADBadTagException, BadPaddingException, ChaCha20, ChaCha20Poly1305, Crypto,  # noqa: F401
                     IllegalStateException, Poly1305)
from .handshake import SymmetricKeypair  # noqa: F401
