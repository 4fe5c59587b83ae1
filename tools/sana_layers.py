"""Shape table of the Sana-Sprint 1.6B LoRA targets for one member at 1024 px (16 images: 16 x 1024
image tokens, 16 x 300 caption tokens, 16 time rows), as hyperscalees_t2i_amd/sana.py builds them
(168 targets).  Diagnostic tools only."""


def sana_lora_layers():
    """[(rows_per_member, K, N, count)]"""
    return [
        (16384, 2240, 2240, 120),  # attn1 to_q/k/v/out, attn2 to_q/out (x20 blocks)
        (4800, 2240, 2240, 40),    # attn2 to_k/v on the caption tokens (x20)
        (4800, 2304, 2240, 1),     # caption_projection.linear_1
        (4800, 2240, 2240, 1),     # caption_projection.linear_2
        (16, 256, 2240, 2),        # time_embed.{timestep,guidance}_embedder.linear_1
        (16, 2240, 2240, 2),       # time_embed.{timestep,guidance}_embedder.linear_2
        (16, 2240, 13440, 1),      # time_embed.linear
        (16384, 2240, 32, 1),      # proj_out
    ]
