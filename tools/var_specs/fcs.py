# FC weight-gradient split count inside the merged FC backward launch (dgrad tiles fixed)
H = "impala.hip"
FC = "  h->spfc = plan_split(N, (FLAT / 256) * (HID / 64), 96);"
VARIANTS = {
    "fcs6": [],
    "fcs8": [(H, FC, FC.replace("96)", "128)"))],
    "fcs12": [(H, FC, FC.replace("96)", "192)"))],
    "fcs4": [(H, FC, FC.replace("96)", "64)"))],
}
