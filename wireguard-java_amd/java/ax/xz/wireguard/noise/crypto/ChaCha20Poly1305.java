package ax.xz.wireguard.noise.crypto;

import javax.crypto.AEADBadTagException;
import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;
import java.util.Arrays;

import static java.lang.foreign.ValueLayout.JAVA_BYTE;
import static java.lang.foreign.ValueLayout.JAVA_INT;

/**
 * Drop-in for ax.xz.wireguard.noise.crypto.ChaCha20Poly1305 (reference
 * ChaCha20Poly1305.java:10-98): same public static API, RFC 8439 AEAD computed on
 * the MI355X by libwgaead. Decrypt verifies first and leaves {@code plaintext}
 * untouched on a bad tag (reference :40-56).
 */
public class ChaCha20Poly1305 {
	public static void poly1305ChaChaKeyGen(MemorySegment chacha20StateBuffer, MemorySegment key, MemorySegment nonce, MemorySegment output) {
		ChaCha20.initializeState(key, nonce, chacha20StateBuffer, 0);
		ChaCha20.chacha20Block(chacha20StateBuffer, output, 0);
	}

	public static byte[] poly1305ChaChaKeyGen(byte[] key, byte[] nonce) {
		try (var arena = Arena.ofConfined()) {
			var state = arena.allocate(64, 16);
			var output = arena.allocate(64, 16);
			poly1305ChaChaKeyGen(state, MemorySegment.ofArray(key), MemorySegment.ofArray(nonce), output);
			return output.asSlice(0, 32).toArray(JAVA_BYTE);
		}
	}

	public static void poly1305AeadEncrypt(MemorySegment key, MemorySegment nonce, MemorySegment plaintext, MemorySegment ciphertext, MemorySegment tag) {
		poly1305AeadEncrypt(null, key, nonce, plaintext, ciphertext, tag);
	}

	public static void poly1305AeadEncrypt(MemorySegment aad, MemorySegment key, MemorySegment nonce, MemorySegment plaintext, MemorySegment ciphertext, MemorySegment tag) {
		long len = plaintext.byteSize();
		try (var arena = Arena.ofConfined()) {
			var out = arena.allocate(len + 16, 16);
			WgAead.aead(WgAead.WG_MODE_SEAL, key, word(nonce, 0), word(nonce, 4), word(nonce, 8), 0, plaintext, aad, out, len);
			ciphertext.copyFrom(out.asSlice(0, len));
			tag.copyFrom(out.asSlice(len, 16));
		}
	}

	public static void poly1305AeadDecrypt(MemorySegment aad, MemorySegment key, MemorySegment nonce, MemorySegment ciphertext, MemorySegment plaintext, MemorySegment tag) throws AEADBadTagException {
		long len = ciphertext.byteSize();
		try (var arena = Arena.ofConfined()) {
			var in = arena.allocate(len + 16, 16);
			in.asSlice(0, len).copyFrom(ciphertext);
			in.asSlice(len, 16).copyFrom(tag.asSlice(0, 16));
			var out = arena.allocate(Math.max(1, len), 16);
			int status = WgAead.aead(WgAead.WG_MODE_OPEN, key, word(nonce, 0), word(nonce, 4), word(nonce, 8), 0, in, aad, out, len);
			if (status != WgAead.WG_PKT_OK)
				throw new AEADBadTagException("Invalid tag (got %s)".formatted(Arrays.toString(tag.toArray(JAVA_BYTE))));
			plaintext.copyFrom(out.asSlice(0, len));
		}
	}

	public static void poly1305AeadDecrypt(MemorySegment key, MemorySegment nonce, MemorySegment ciphertext, MemorySegment plaintext, MemorySegment tag) throws AEADBadTagException {
		poly1305AeadDecrypt(null, key, nonce, ciphertext, plaintext, tag);
	}

	static int word(MemorySegment nonce, long off) {
		return nonce.get(JAVA_INT.withByteAlignment(1), off);
	}
}
